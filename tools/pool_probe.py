"""k_dsmp A/B aid: a resident 2^20 batch through the per-lane (k_dsm) and the
pooled (k_ai + k_dsmp + k_fin) double-scalar multiply, DSM-stage time from
HIP events, verdicts compared, and the pool's fill statistics when the
library was built with FD_AMD_DIAG (fd_amd_pool_debug)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from firedancer_amd import ed25519, hip, workload  # noqa: E402

n = int(os.environ.get("N", 1 << 20))
pub, sig, off, sz, blob = workload.sig_batch(n, 200, 5)
d = {k: hip.DeviceBuffer.from_array(v) for k, v in dict(pub=pub, sig=sig, off=off, sz=sz, blob=blob).items()}
d_err = hip.DeviceBuffer(n)
d_ws = hip.DeviceBuffer(ed25519.workspace_footprint(n))
st = hip.Stream()
L = ed25519.lib()
try:
    dbg = L.fd_amd_pool_debug
except AttributeError:
    dbg = None


def run(ev=None):
    ed25519.verify_dev_ev(n, d["pub"].ptr, d["sig"].ptr, d["off"].ptr, d["sz"].ptr, d["blob"].ptr, d_err.ptr,
                          d_ws.ptr, st.handle, ev)


res = {"lib": os.path.basename(ed25519.LIB_PATH), "n": n, "waves": os.environ.get("FD_POOL_WAVES")}
ref = None
for kern in ("k_dsm", "k_dsmp"):
    ed25519.select_dsm_kernel(kern)
    run()
    st.synchronize()
    err = d_err.to_array(np.int8, n)
    if ref is None:
        ref = err
    ms = []
    for _ in range(3):
        if dbg:
            buf = (ctypes.c_uint * 4)()
            dbg(buf, 1)
        ev = [hip.Event() for _ in range(4)]
        run(ev)
        st.synchronize()
        ms.append(ev[2].elapsed_ms(ev[3]))
    res[kern] = {"dsm_ms": min(ms), "same": bool(np.array_equal(err, ref))}
    if kern == "k_dsmp" and dbg:
        buf = (ctypes.c_uint * 4)()
        dbg(buf, 0)
        steps, lanes, add, idle = list(buf)
        res["pool"] = {"steps": steps, "fill": lanes / max(1, 64 * steps), "add_frac": add / max(1, steps),
                       "idle": idle}
        tb = np.zeros((8192, 4), np.uint64)
        if L.fd_amd_pool_debug_times(ctypes.c_void_p(tb.ctypes.data)) == 0:
            W = int(os.environ.get("FD_POOL_WAVES") or 2048)
            t = tb[:W, :3].astype(np.float64)
            t0 = t[:, 0].min()
            f = 100e6 / 1e3   # wall_clock64 ticks per ms (100 MHz)
            st, te, en = (t[:, 0] - t0) / f, (t[:, 1] - t0) / f, (t[:, 2] - t0) / f
            sa = (tb[:W, 3] & 0xffffffff).astype(np.float64)
            la = (tb[:W, 3] >> 32).astype(np.float64)
            q = lambda a: [round(float(np.percentile(a, x)), 3) for x in (0, 10, 50, 90, 100)]
            res["waves_ms"] = {"start": q(st), "exhausted": q(te), "end": q(en), "drain": q(en - te),
                               "steps_after": q(sa), "fill_after": float(la.sum() / max(1.0, 64 * sa.sum())),
                               "avg_resident": float((en - st).sum() / en.max())}
ed25519.select_dsm_kernel("default")
print(json.dumps(res), flush=True)

"""k_dsm4 time vs batch size (inputs resident, latency kernels forced):
separates one wave's serial op-stream time (4096: one wave per CU; 16384:
one per SIMD) from issue contention (more waves per SIMD)."""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
from firedancer_amd import ed25519, hip, workload  # noqa: E402

ed25519.select_dsm_kernel(os.environ.get("FD_DSM_KERNEL", "k_dsm4"))
for n in (1024, 4096, 16384, 32768, 65536, 131072):
    pub, sig, off, sz, blob = workload.sig_batch(n, 200, 5)
    d = {k: hip.DeviceBuffer.from_array(v) for k, v in dict(pub=pub, sig=sig, off=off, sz=sz, blob=blob).items()}
    err = hip.DeviceBuffer(n); ws = hip.DeviceBuffer(ed25519.workspace_footprint(n)); st = hip.Stream()
    t = np.zeros(3)
    for r in range(6):
        ev = [hip.Event() for _ in range(4)]
        ed25519.verify_dev_ev(n, d["pub"].ptr, d["sig"].ptr, d["off"].ptr, d["sz"].ptr, d["blob"].ptr, err.ptr, ws.ptr,
                              st.handle, ev)
        st.synchronize()
        if r >= 1:
            t += [ev[j].elapsed_ms(ev[j + 1]) for j in range(3)]
    t /= 5
    waves = (n + 15) // 16
    print(json.dumps({"n": n, "waves": waves, "waves_per_simd": waves / 1024.0, "k_front_ms": t[0],
                      "k_dsm4_ms": t[2], "k_dsm4_us_per_wave_round": t[2] * 1e3 / max(1.0, waves / 1024.0)}))

"""Per-batch GPU latency floor: verify_dev_ev stage times for small batches
(inputs resident, one batch at a time)."""
import os, sys, json
sys.path.insert(0, os.getcwd())
import numpy as np
from firedancer_amd import ed25519, hip
rng = np.random.default_rng(1)
res = {}
for n in (64, 256, 1024, 4096, 16384, 65536):
    prv = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    blob = rng.integers(0, 256, n * 200 + 1, dtype=np.uint8)
    off = (np.arange(n) * 200).astype(np.uint32); sz = np.full(n, 200, np.uint32)
    pub, sig = ed25519.sign_batch(prv, blob, off, sz)
    d = {k: hip.DeviceBuffer.from_array(v) for k, v in dict(pub=pub, sig=sig, off=off, sz=sz, blob=blob).items()}
    err = hip.DeviceBuffer(n); ws = hip.DeviceBuffer(ed25519.workspace_footprint(n)); st = hip.Stream()
    t = np.zeros(3)
    for r in range(6):
        ev = [hip.Event() for _ in range(4)]
        ed25519.verify_dev_ev(n, d["pub"].ptr, d["sig"].ptr, d["off"].ptr, d["sz"].ptr, d["blob"].ptr, err.ptr, ws.ptr, st.handle, ev)
        st.synchronize()
        if r >= 1:
            t += [ev[j].elapsed_ms(ev[j + 1]) for j in range(3)]
    t /= 5
    res[n] = {"k_prep": t[0], "k_decomp": t[1], "k_dsm": t[2], "total_ms": t.sum()}
    print(n, json.dumps(res[n]))

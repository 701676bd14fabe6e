import sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np
from firedancer_amd import ed25519, hip, workload
n = 64
pub, sig, off, sz, blob = workload.sig_batch(n, 200, 1)
K = 4
bufs = []
for k in range(K):
    d = {kk: hip.DeviceBuffer.from_array(v) for kk, v in dict(pub=pub, sig=sig, off=off, sz=sz, blob=blob).items()}
    bufs.append((d, hip.DeviceBuffer(n), hip.DeviceBuffer(ed25519.workspace_footprint(n)), hip.Stream()))
def go(m):
    t0 = time.perf_counter()
    for k in range(m):
        d, e, w, s = bufs[k]
        ed25519.verify_dev(n, d["pub"].ptr, d["sig"].ptr, d["off"].ptr, d["sz"].ptr, d["blob"].ptr, e.ptr, w.ptr, s.handle)
    for k in range(m):
        bufs[k][3].synchronize()
    return (time.perf_counter() - t0) * 1e3
for m in (1, 2, 4, 1, 2, 4):
    print(m, "batches on", m, "streams: %.3f ms" % go(m))

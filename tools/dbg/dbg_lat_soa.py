"""Host-batch latency path (verify_soa of 4096) for a kernel+copy trace."""
import os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np
from firedancer_amd import ed25519, workload
n = 4096
pub, sig, off, sz, blob = workload.sig_batch(n, 200, 7)
eng = ed25519.Engine(device=0, batch_max=n, blob_max=n * 200)
lat = []
for r in range(30):
    t = time.perf_counter(); eng.verify_soa(pub, sig, off, sz, blob); lat.append((time.perf_counter() - t) * 1e3)
print("p50 %.3f ms" % np.percentile(lat[5:], 50))

"""Host-SoA throughput sweep: slots in flight x chunk size (PCIe-inclusive path)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np
from firedancer_amd import ed25519, workload

n = 1 << 20
pub, sig, off, sz, blob = workload.sig_batch(n, 200, 1000)
for nslot in (2, 3, 4):
    os.environ["FD_ED25519_AMD_NSLOT"] = str(nslot)
    for chunk in (1 << 16, 1 << 17, 1 << 18):
        eng = ed25519.Engine(device=0, batch_max=chunk, blob_max=chunk * 200)
        eng.verify_soa(pub[:chunk], sig[:chunk], off[:chunk], sz[:chunk], blob)
        t = time.perf_counter()
        for _ in range(3):
            eng.verify_soa(pub, sig, off, sz, blob)
        dt = (time.perf_counter() - t) / 3
        eng.close()
        print("nslot %d chunk %7d  %.1f M/s" % (nslot, chunk, n / dt / 1e6), flush=True)

"""PCIe-inclusive host paths (A/B aid): 2^20 x 200-B signatures handed over as
host SoA, staged (verify_soa) and registered (verify_soa_registered), per
engine chunk size and chunks in flight (FD_ED25519_AMD_NSLOT)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
import numpy as np  # noqa: E402
from firedancer_amd import ed25519, workload  # noqa: E402

n = 1 << 20
pub, sig, off, sz, blob = workload.sig_batch(n, 200, 11)
reg = ed25519.RegisteredPlanes(pub, sig, off, sz, blob)
ref = None
for nslot in (2, 3, 4):
    os.environ["FD_ED25519_AMD_NSLOT"] = str(nslot)
    for lg in (16, 17, 18):
        chunk = 1 << lg
        eng = ed25519.Engine(device=0, batch_max=chunk, blob_max=chunk * 200)
        err = np.zeros(n, np.int8)
        eng.verify_soa_registered(reg[0], reg[1], reg[2], reg[3], reg[4], err)
        if ref is None:
            ref = err.copy()
        t = []
        for _ in range(4):
            t0 = time.perf_counter()
            eng.verify_soa_registered(reg[0], reg[1], reg[2], reg[3], reg[4], err)
            t.append(time.perf_counter() - t0)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            e2 = eng.verify_soa(pub, sig, off, sz, blob)
            ts.append(time.perf_counter() - t0)
        eng.close()
        print(json.dumps({"nslot": nslot, "chunk": chunk, "registered_Mps": n / min(t) / 1e6,
                          "staged_Mps": n / min(ts) / 1e6, "ok": bool((err == ref).all() and (e2 == ref).all())}))
reg.close()

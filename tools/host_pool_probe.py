"""Registered host path (fd_ed25519_amd_verify_soa_registered, 2^20 x 200 B)
with the per-lane k_dsm vs the pooled k_dsmp on the engine's chunks (A/B
aid): chunk 2^17..2^19, 2 chunks in flight, pool threshold lowered to the
chunk size for the pooled rows."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
from firedancer_amd import ed25519, workload  # noqa: E402

n = 1 << 20
pub, sig, off, sz, blob = workload.sig_batch(n, 200, 11)
reg = ed25519.RegisteredPlanes(pub, sig, off, sz, blob)
ref = None
for lg in (17, 18, 19):
    chunk = 1 << lg
    for pooled in (False, True):
        ed25519.set_pool_batch_min(chunk if pooled else 1 << 19)
        if not pooled and lg == 19:
            ed25519.set_pool_batch_min(1 << 20)
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
        print(json.dumps({"chunk": chunk, "pooled": pooled, "verifies_per_s": n / min(t),
                          "same": bool(np.array_equal(err, ref))}), flush=True)
        eng.close()
ed25519.set_pool_batch_min(1 << 19)

"""Several verify tiles sharing one GPU (the reference scales the verify
stage by running N tiles, src/app/frank/fd_frank_init:67-80): T concurrent
producer -> tile -> consumer pipelines from Python threads (ctypes drops the
GIL in the calls), each its own engine and 4 streams, saturated, every
published frag checked.  Prints one JSON line per tile count."""
import hashlib
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["GPU_MAX_HW_QUEUES"] = str(max(16, int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))))
import numpy as np  # noqa: E402
from firedancer_amd import ed25519, tango, workload  # noqa: E402

m = 1 << 16
pub, sig, off, sz, blob = workload.sig_batch(m, 200, 77)
off = off.astype(np.uint32)
eng = ed25519.Engine(device=0, batch_max=m, blob_max=blob.size + 64)
err = eng.verify_soa(pub, sig, off, sz, blob)
eng.close()
tag = np.array([int.from_bytes(hashlib.sha512(bytes(sig[i][:32]) + bytes(pub[i]) +
                                              bytes(blob[off[i]:off[i] + sz[i]])).digest()[:8], "little")
                for i in range(m)], np.uint64)
frags = int(os.environ.get("FRAGS", 1 << 20))
bmax = int(os.environ.get("BATCH_MAX", 16384))
for T in [int(x) for x in os.environ.get("TILES", "1 2 3").split()]:
    for zc in (True, False):
        res = [None] * T

        def go(k):
            res[k] = tango.bench_stream(0, bmax, 0, pub, sig, off, sz, blob, frags, zero_copy=zc, expect_err=err,
                                        expect_tag=tag, sample_bytes=True)
        th = [threading.Thread(target=go, args=(k,)) for k in range(T)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        wall = time.perf_counter() - t0
        print(json.dumps({"tiles": T, "zero_copy": zc, "batch_max": bmax, "frags_per_tile": frags,
                          "wall_s_incl_setup": wall,
                          "sum_of_tile_rates": sum(r["frags_per_s"] for r in res),
                          "per_tile_frags_per_s": [r["frags_per_s"] for r in res],
                          "mismatches": int(sum(r["mismatches"] for r in res)),
                          "checked": int(sum(r["checked"] for r in res))}), flush=True)

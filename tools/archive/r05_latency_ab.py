"""Latency A/B of the 4096-signature host batch (the BASELINE metric's p50):
interleaved rounds over libraries, each round timing `calls` batches from
registered caller memory (fd_ed25519_amd_verify_soa_registered) and from
plain host arrays (fd_ed25519_amd_verify_soa, packed pinned staging).
Every verdict is checked against the first library's.
usage: python tools/r05_latency_ab.py OUT.jsonl LIB[,LIB...] [rounds] [calls]
       LIB "" = the product library; each library runs in its own process."""
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib, calls, out):
    if lib:
        os.environ["FD_AMD_LIB"] = os.path.join(ROOT, lib)
    sys.path.insert(0, ROOT)
    from firedancer_amd import ed25519, workload
    n, m, sz = 1 << 16, 4096, 200
    pub, sig, off, szs, blob = workload.sig_batch(n, sz, 4242)
    eng = ed25519.Engine(device=0, batch_max=m, blob_max=m * sz)
    reg = ed25519.RegisteredPlanes(pub, sig, off, szs, blob)
    rerr = np.zeros(m, np.int8)
    b_off = (np.arange(m, dtype=np.uint32) * sz).astype(np.uint32)
    res = {"lib": lib or "product"}
    for way in ("registered", "staged"):
        lat, errs = [], []
        for r in range(calls + 10):
            lo = (r * m) % (n - m)
            t1 = time.perf_counter()
            if way == "registered":
                eng.verify_soa_registered(reg[0][lo:lo + m], reg[1][lo:lo + m], reg[2][lo:lo + m], reg[3][lo:lo + m],
                                          reg[4], rerr)
                e = rerr.copy()
            else:
                e = eng.verify_soa(pub[lo:lo + m], sig[lo:lo + m], b_off, szs[lo:lo + m],
                                   blob[off[lo]:off[lo] + m * sz])
            dt = (time.perf_counter() - t1) * 1e6
            if r >= 10:
                lat.append(dt)
            errs.append(int(e.astype(np.int64).sum()))
        lat = np.array(lat)
        res[way] = {"p50_us": float(np.percentile(lat, 50)), "p99_us": float(np.percentile(lat, 99)),
                    "min_us": float(lat.min()), "verdict_sums": errs[:5]}
    reg.close()
    eng.close()
    with open(out, "a") as f:
        f.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]), sys.argv[4])
        sys.exit(0)
    out, libs = sys.argv[1], sys.argv[2].split(",")
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    calls = int(sys.argv[4]) if len(sys.argv) > 4 else 300
    for r in range(rounds):
        for lib in libs:
            rc = subprocess.call([sys.executable, os.path.abspath(__file__), "--child", lib, str(calls), out],
                                 timeout=300)
            if rc:
                sys.exit(rc)

"""Interleaved A/B of the streaming tile's saturated rows between libraries:
each round runs every library in its own process over the same pool (2^16
frags of 200-B messages, 10 % with one flipped message bit), saturated, every
published frag checked against the batch engine's verdicts and the SHA-512
tags.  Reports whole-run and steady rates and the mean fill of throughput
chunks (frags per 64-lane chunk).
usage: python tools/r05_tile_ab.py OUT.jsonl LIB[,LIB...] [rounds] [frags] [bmax,...]
       LIB "" = the product library; NAME=VALUE = the product library with that
       environment variable set (e.g. FD_AMD_BENCH_WINDOW=524288)."""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib, frags, bmaxes, out):
    if "=" in lib:      # NAME=VALUE: the product library with that environment variable set
        k, v = lib.split("=", 1)
        os.environ[k] = v
    elif lib:
        os.environ["FD_AMD_LIB"] = os.path.join(ROOT, lib)
    sys.path.insert(0, ROOT)
    from firedancer_amd import ed25519, tango, workload
    m = 1 << 16
    pub, sig, off, sz, blob = workload.sig_batch(m, 200, 77)
    rng = np.random.default_rng(55)
    for i in rng.choice(m, m // 10, replace=False):
        blob[off[i] + int(rng.integers(0, 200))] ^= 1 << int(rng.integers(0, 8))
    eng = ed25519.Engine(device=0, batch_max=m, blob_max=blob.size + 64)
    err = eng.verify_soa(pub, sig, off, sz, blob)
    eng.close()
    tag = np.array([int.from_bytes(hashlib.sha512(bytes(sig[i][:32]) + bytes(pub[i]) +
                                                  bytes(blob[off[i]:off[i] + sz[i]])).digest()[:8], "little")
                    for i in range(m)], np.uint64)
    res = {"lib": lib or "product", "rows": []}
    for bmax in bmaxes:
        for zc in (True, False):
            r = tango.bench_stream(0, bmax, 0, pub, sig, off, sz, blob, frags, zero_copy=zc, expect_err=err,
                                   expect_tag=tag, sample_bytes=True)
            res["rows"].append({"bmax": bmax, "mode": "zero_copy" if zc else "copy",
                                "sat": round(r["frags_per_s"] / 1e6, 2), "steady": round(r["steady_frags_per_s"] / 1e6, 2),
                                "fill": round(r["gpu_frags_thr"] / max(r["gpu_chunks_thr"], 1.0), 1),
                                "hand_offs": int(r["hand_offs"]), "stop_window": int(r["stop_window"]),
                                "ok": int(r["mismatches"]) == 0 and int(r["checked"]) > 0})
    with open(out, "a") as f:
        f.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]), [int(x) for x in sys.argv[4].split(",")], sys.argv[5])
        sys.exit(0)
    out, libs = sys.argv[1], sys.argv[2].split(",")
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    frags = int(sys.argv[4]) if len(sys.argv) > 4 else 1 << 22
    bm = sys.argv[5] if len(sys.argv) > 5 else "1024,16384"
    for r in range(rounds):
        for lib in libs:
            rc = subprocess.call([sys.executable, os.path.abspath(__file__), "--child", lib, str(frags), bm, out],
                                 timeout=300)
            if rc:
                sys.exit(rc)

"""Interleaved A/B of library builds on the streaming tile: saturated runs
checked frag by frag (the bench's configs[4] pool: 2^16 signatures of 200 B,
10 % with a flipped message bit) at zero copy 4096 / 16384 and copy 16384,
plus paced runs at fixed offered rates (zero copy 4096).  Each build runs in
its own process (FD_AMD_LIB); one JSON line per run.

usage: python tools/tile_lib_ab.py <rounds> <frags> lib1.so [lib2.so ...]   (a lib "-" = the product;
       "-@VAR=val;VAR2=val2" = the product with those environment variables)
env: AB_RATES="27e6, 43e6" paced rates (empty: none), AB_SAT="((4096, True),)" saturated (batch_max, zero copy)
     runs, AB_PACED="((4096, True),)" the paced runs' (batch_max, zero copy), AB_SECS=0.4 their length,
     AB_CONTINUE=1 records a failing build and goes on (an experiment's control)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import hashlib, json, os, sys
sys.path.insert(0, %(root)r)
import numpy as np
import bench
from firedancer_amd import ed25519, tango
frags = %(frags)d
m = 1 << 16
pub, sig, off, sz, blob = bench.make_workload(m, 200, 7)
off = (off - off[0]).astype(np.uint32)
rng = np.random.default_rng(55)
for i in rng.choice(m, m // 10, replace=False):
    blob[off[i] + int(rng.integers(0, int(sz[i])))] ^= 1 << int(rng.integers(0, 8))
eng = ed25519.Engine(device=0, batch_max=m, blob_max=blob.size + 64)
err = eng.verify_soa(pub, sig, off, sz, blob)
eng.close()
tag = np.array([int.from_bytes(hashlib.sha512(bytes(sig[i][:32]) + bytes(pub[i]) +
                bytes(blob[off[i]:off[i] + sz[i]])).digest()[:8], "little") for i in range(m)], np.uint64)
pool = (pub, sig, off, sz, blob)
out = []
for bmax, zc in %(sat)s:
    r = tango.bench_stream(0, bmax, 0, *pool, frags, zero_copy=zc, expect_err=err, expect_tag=tag, sample_bytes=True)
    out.append({"kind": "sat", "bmax": bmax, "zc": zc, "mfps": round(r["frags_per_s"] / 1e6, 2),
                "steady_mfps": round(r["steady_frags_per_s"] / 1e6, 2), "mismatches": int(r["mismatches"]),
                "chunks": [int(r["gpu_chunks_lat"]), int(r.get("gpu_chunks_quad", 0)), int(r["gpu_chunks_thr"])],
                "stager_ns": [round(r.get(k, 0.0), 2) for k in ("stager_list_ns", "stager_copy_ns", "stager_stage_ns",
                                                                  "stager_hand_ns")]})
for bmax, zc in %(paced)s:
    for rate in (%(rates)s):
        r = tango.bench_stream(0, bmax, 0, *pool, int(rate * %(secs)s), rate=rate, zero_copy=zc)
        out.append({"kind": "paced", "bmax": bmax, "zc": zc, "offered_m": rate / 1e6, "p50_us": round(r["p50_ns"] / 1e3, 1),
                    "p99_us": round(r["p99_ns"] / 1e3, 1), "switches": int(r["mode_switches"]),
                    "chunks": [int(r["gpu_chunks_lat"]), int(r.get("gpu_chunks_quad", 0)), int(r["gpu_chunks_thr"])],
                    "stalls_us": [round(r[k] / 1e3, 1) for k in ("producer_late_max_ns", "tile_pass_max_ns",
                                                                  "consumer_gap_max_ns")]})
print(json.dumps(out))
'''

if __name__ == "__main__":
    rounds, frags, libs = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3:]
    rates = os.environ.get("AB_RATES", "27e6, 43e6")
    for r in range(rounds):
        for lib in libs:
            env = dict(os.environ)
            if lib.startswith("-@"):
                env.update(kv.split("=", 1) for kv in lib[2:].split(";") if kv)
            elif lib != "-":
                env["FD_AMD_LIB"] = os.path.abspath(lib)
            sat = os.environ.get("AB_SAT", "((4096, True), (16384, True), (16384, False))")
            paced = os.environ.get("AB_PACED", "((4096, True),)")
            secs = float(os.environ.get("AB_SECS", "0.4"))
            p = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT, "frags": frags, "rates": rates, "sat": sat,
                                                               "paced": paced, "secs": secs}],
                               env=env, capture_output=True, text=True, timeout=300)
            if p.returncode:
                print(json.dumps({"round": r, "lib": lib, "rc": p.returncode, "err": p.stderr[-800:]}), flush=True)
                if os.environ.get("AB_CONTINUE"):   # a build expected to fail (an experiment's control)
                    continue
                sys.exit(1)
            for x in json.loads(p.stdout.strip().splitlines()[-1]):
                x.update(round=r, lib=lib)
                print(json.dumps(x), flush=True)

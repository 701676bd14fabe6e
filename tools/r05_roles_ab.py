"""Interleaved A/B of the tile kernel's wave roles (FD_AMD_TILE_ROLES=1: a
SIMD's second wave claims only descriptors no wave waits for; 0: every wave
takes tickets as it goes idle).  Each round runs both settings in their own
process: a saturated run (every frag checked), then paced runs at 50 % and
80 % of that run's rate, zero copy; JSON lines with the rate, p50 / p99,
the service / queue / publish-wait tails and the second waves' share.
Runs against commit 8857e83 (the roles code was removed after it; profiles/r05_tile_roles_ab.txt).
usage: python tools/r05_roles_ab.py OUT.jsonl [rounds] [bmax,...] [paced_seconds]"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(roles, bmaxes, secs, out):
    os.environ["FD_AMD_TILE_ROLES"] = roles
    sys.path.insert(0, ROOT)
    from firedancer_amd import ed25519, tango, workload
    m = 1 << 16
    pub, sig, off, sz, blob = workload.sig_batch(m, 200, 77)
    eng = ed25519.Engine(device=0, batch_max=m, blob_max=blob.size + 64)
    err = eng.verify_soa(pub, sig, off, sz, blob)
    eng.close()
    tag = np.array([int.from_bytes(hashlib.sha512(bytes(sig[i][:32]) + bytes(pub[i]) +
                                                  bytes(blob[off[i]:off[i] + sz[i]])).digest()[:8], "little")
                    for i in range(m)], np.uint64)
    pool = (pub, sig, off, sz, blob)
    for bmax in bmaxes:
        sat = tango.bench_stream(0, bmax, 0, *pool, 1 << 22, zero_copy=True, expect_err=err, expect_tag=tag,
                                 sample_bytes=True)
        rows = [{"load": "sat", "frags_per_s": round(sat["frags_per_s"] / 1e6, 2),
                 "ok": int(sat["mismatches"]) == 0 and int(sat["checked"]) > 0,
                 "second_waves": int(sat["second_waves"]), "second_chunks": int(sat["second_chunks"]),
                 "chunks": int(sat["gpu_chunks_lat"] + sat["gpu_chunks_thr"])}]
        for f in (0.5, 0.8):
            rate = f * sat["frags_per_s"]
            r = tango.bench_stream(0, bmax, 0, *pool, int(rate * secs), rate=rate, zero_copy=True)
            rows.append({"load": f, "p50_us": round(r["p50_ns"] / 1e3, 1), "p99_us": round(r["p99_ns"] / 1e3, 1),
                         "x": round(r["p99_ns"] / max(r["p50_ns"], 1.0), 2),
                         "service_us": [round(r["service_p50_ns"] / 1e3, 1), round(r["service_p99_ns"] / 1e3, 1)],
                         "queue_p99_us": round(r["queue_p99_ns"] / 1e3, 1),
                         "publish_p99_us": round(r["publish_p99_ns"] / 1e3, 1),
                         "input_p99_us": round(r["input_p99_ns"] / 1e3, 1),
                         "second_chunks": int(r["second_chunks"]),
                         "chunks": int(r["gpu_chunks_lat"] + r["gpu_chunks_thr"])})
        with open(out, "a") as fo:
            fo.write(json.dumps({"roles": roles, "bmax": bmax, "rows": rows}) + "\n")


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2], [int(x) for x in sys.argv[3].split(",")], float(sys.argv[4]), sys.argv[5])
        sys.exit(0)
    out = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    bm = sys.argv[3] if len(sys.argv) > 3 else "4096,16384"
    secs = sys.argv[4] if len(sys.argv) > 4 else "0.5"
    for _ in range(rounds):
        for roles in ("1", "0"):
            rc = subprocess.call([sys.executable, os.path.abspath(__file__), "--child", roles, bm, secs, out],
                                 timeout=300)
            if rc:
                sys.exit(rc)

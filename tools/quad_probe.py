"""Quad chunks (16 frags, k_dsm4's body) on the streaming tile: their
saturated capacity with every chunk forced to each level, and the AUTO rule's
latency at fixed offered rates -- the numbers the tile's quad thresholds
(fd_verify_tile.cpp QUAD_SVC_S, rate_hi/lo) are set from.  One JSON line per
run.

usage: python tools/quad_probe.py [sat|paced|all] > gpurun_out/quad_probe.jsonl
env FD_AMD_BENCH_LEVELS="quad_hi,quad_lo,thr_hi,thr_lo" overrides the level thresholds (slots/s);
QP_PAIRS="0,1" runs every line with quad pairs off and on (FD_AMD_TILE_PAIRS, read per tile).
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from firedancer_amd import ed25519, tango  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "all"
rates = [float(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [10e6, 15e6, 20e6, 25e6, 28e6, 30e6, 32e6, 35e6]
m = 1 << 16
pub, sig, off, sz, blob = bench.make_workload(m, 200, 7)
off = (off - off[0]).astype(np.uint32)
pool = (pub, sig, off, sz, blob)
eng = ed25519.Engine(device=0, batch_max=m, blob_max=blob.size + 64)
err = eng.verify_soa(*pool)
eng.close()
names = {0: "auto", 1: "latency", 2: "throughput", 3: "quad"}


def line(**kw):
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in kw.items()}), flush=True)


def keep(r):
    return {"frags_per_s": r["frags_per_s"], "steady": r["steady_frags_per_s"], "p50_us": r["p50_ns"] / 1e3,
            "p99_us": r["p99_ns"] / 1e3, "service_p50_us_lat_quad": r["service_lat_chunk_p50_ns"] / 1e3,
            "service_p50_us_thr": r["service_thr_chunk_p50_ns"] / 1e3, "queue_p50_us": r["queue_p50_ns"] / 1e3,
            "chunks": [int(r["gpu_chunks_lat"]), int(r["gpu_chunks_quad"]), int(r["gpu_chunks_thr"])],
            "switches": int(r["mode_switches"]), "mismatches": int(r["mismatches"]),
            "stager_ns": [round(r[k], 1) for k in ("stager_list_ns", "stager_copy_ns", "stager_stage_ns", "stager_hand_ns")],
            "quad_pairs": int(r.get("quad_pairs", 0)), "pairs_env": os.environ.get("FD_AMD_TILE_PAIRS", "0")}


pair_set = os.environ.get("QP_PAIRS", os.environ.get("FD_AMD_TILE_PAIRS", "0")).split(",")


def bench_stream(*a, **kw):
    """tango.bench_stream once per QP_PAIRS setting; yields the results."""
    for ps in pair_set:
        os.environ["FD_AMD_TILE_PAIRS"] = ps
        yield tango.bench_stream(*a, **kw)


if what in ("sat", "all"):
    for bmax in (1024, 4096):
        for mode in (1, 3, 2):
            for r in bench_stream(0, bmax, 0, *pool, 1 << 22, zero_copy=True, chunk_mode=mode):
                line(kind="saturated", bmax=bmax, mode=names[mode], **keep(r))
    for zc in (False, True):   # AUTO, both stagings: the stager's time per frag by phase
        for r in bench_stream(0, 4096, 0, *pool, 1 << 22, zero_copy=zc):
            line(kind="saturated", bmax=4096, mode="auto", staging="zero_copy" if zc else "copy", **keep(r))
if what in ("paced", "all"):
    for bmax in (4096,):
        for rate in rates:
            for mode in (0, 3):
                nf = int(max(50000, rate * 0.3))
                for r in bench_stream(0, bmax, 0, *pool, nf, rate=rate, zero_copy=True, chunk_mode=mode):
                    line(kind="paced", bmax=bmax, mode=names[mode], offered=rate, **keep(r))

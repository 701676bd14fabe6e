"""Tile A/B: batches in flight (FD_AMD_TILE_NSLOT) x kernel policy
(FD_AMD_TILE_TPUT_MIN / _NFLY: large batches launched while others are in
flight take the 1-lane kernel).  Saturated rate and p50/p99 at 50 % / 80 %
load, zero-copy staging."""
import sys, os
sys.path.insert(0, os.getcwd())
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("GPU_MAX_HW_QUEUES", "16")
from firedancer_amd import tango, workload
pub, sig, off, sz, blob = workload.sig_batch(65536, 200, 1)
grid = [tuple(int(v) for v in g.split(":")) for g in os.environ.get("GRID", "4:0:2,6:0:2,8:0:2").split(",")]
import itertools
for bmax, (nslot, tmin, nfly) in itertools.product([int(x) for x in os.environ.get("BMAX", "1024,4096,16384").split(",")], grid):
    if 1:
        os.environ["FD_AMD_TILE_NSLOT"] = str(nslot)
        os.environ["FD_AMD_TILE_TPUT_MIN"] = str(tmin)
        os.environ["FD_AMD_TILE_TPUT_NFLY"] = str(nfly)
        r = tango.bench_stream(0, bmax, 0, pub, sig, off, sz, blob, 1 << 20, zero_copy=True)
        r2 = tango.bench_stream(0, bmax, 0, pub, sig, off, sz, blob, 1 << 19, rate=0.5 * r["frags_per_s"], zero_copy=True)
        r3 = tango.bench_stream(0, bmax, 0, pub, sig, off, sz, blob, 1 << 19, rate=0.8 * r["frags_per_s"], zero_copy=True)
        print("zc bmax %5d nslot %2d tput_min %5d nfly %d: sat %.2f M/s batch %.0f | @50%%: p50 %.2f p99 %.2f ms | "
              "@80%%: p50 %.2f p99 %.2f ms" % (bmax, nslot, tmin, nfly, r["frags_per_s"] / 1e6, r["mean_batch"],
                                              r2["p50_ns"] / 1e6, r2["p99_ns"] / 1e6, r3["p50_ns"] / 1e6, r3["p99_ns"] / 1e6),
              flush=True)

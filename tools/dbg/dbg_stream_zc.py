import sys, os, json
sys.path.insert(0, os.getcwd())
os.environ["GPU_MAX_HW_QUEUES"] = "8"
import numpy as np
from firedancer_amd import tango, workload
pub, sig, off, sz, blob = workload.sig_batch(65536, 200, 1)
for zc in (False, True):
    for bmax in (1024, 4096, 16384):
        r = tango.bench_stream(0, bmax, 0, pub, sig, off, sz, blob, 1 << 19, zero_copy=zc)
        r2 = tango.bench_stream(0, bmax, 0, pub, sig, off, sz, blob, 1 << 18, rate=0.5 * r["frags_per_s"], zero_copy=zc)
        print("zc" if zc else "cp", bmax, "sat %.2f M/s batch %.0f" % (r["frags_per_s"] / 1e6, r["mean_batch"]),
              "| @50%%: p50 %.2f ms p99 %.2f ms" % (r2["p50_ns"] / 1e6, r2["p99_ns"] / 1e6), flush=True)

"""Copy-mode tail probe: one saturated run, then REPEATS paced runs at FRAC
of its rate (copy mode, 200-B frags), each printed as a JSON line with its
p50 / p99, the latency decomposition's p99s, the host stall clocks, the run
loop's stop counters and the copy helper's steals -- to find which stop
holds staging when input wait reaches ms.
usage: python tools/r05_copy_tail_probe.py BATCH_MAX [repeats] [frac] [seconds]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd import tango, workload  # noqa: E402

bmax = int(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
frac = float(sys.argv[3]) if len(sys.argv) > 3 else 0.5
secs = float(sys.argv[4]) if len(sys.argv) > 4 else 0.5
m = 1 << 16
pool = workload.sig_batch(m, 200, 77)
sat = tango.bench_stream(0, bmax, 0, *pool, 1 << 22, zero_copy=False)
print(json.dumps({"saturated_frags_per_s": round(sat["frags_per_s"])}), flush=True)
rate = frac * sat["frags_per_s"]
keys = ("passes", "hand_offs", "stop_window", "stop_frames", "stop_batch_max", "stop_pass_bound", "copy_steals",
        "producer_late_max_ns", "tile_pass_max_ns", "consumer_gap_max_ns")
for i in range(reps):
    r = tango.bench_stream(0, bmax, 0, *pool, int(rate * secs), rate=rate, zero_copy=False)
    print(json.dumps({"run": i, "p50_us": round(r["p50_ns"] / 1e3, 1), "x": round(r["p99_ns"] / max(r["p50_ns"], 1), 2),
                      "p99_us": {k: round(r[k + "_p99_ns"] / 1e3, 1) for k in ("cut", "queue", "service", "publish", "input")},
                      **{k: int(r[k]) for k in keys}}), flush=True)

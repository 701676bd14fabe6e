"""Saturated streaming-tile runs without the consumer's check, so the
per-frag trace (cut / queue / service / publish / input) is on: where a
saturated frag's time goes, and how the rate moves with the run length.
    python tools/r04_sat_probe.py [frag_cnt ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd import tango, workload  # noqa: E402

pool = workload.sig_batch(1 << 16, 200, 9)
counts = [int(a) for a in sys.argv[1:]] or [1 << 20, 1 << 22]
for bmax, zc in ((16384, True), (16384, False), (4096, True)):
    for n in counts:
        r = tango.bench_stream(0, bmax, 0, *pool, n, zero_copy=zc)
        keep = ("frags_per_s", "p50_ns", "p99_ns", "cut_p50_ns", "queue_p50_ns", "queue_p99_ns", "service_p50_ns",
                "service_p99_ns", "publish_p50_ns", "publish_p99_ns", "input_p50_ns", "input_p99_ns",
                "service_thr_chunk_p50_ns", "service_lat_chunk_p50_ns", "gpu_chunks_lat", "gpu_chunks_thr",
                "passes", "stop_window", "stop_pass_bound", "mode_switches")
        print(json.dumps(dict(batch_max=bmax, zero_copy=zc, frags=n, **{k: round(r[k]) for k in keep})), flush=True)

"""batch_max 256 zero copy at 50 / 80 % of its own saturated rate, with the
default window (2^15) or FD_AMD_BENCH_WINDOW's: one child process per
setting, interleaved; JSON lines with the saturated rate, the chunk modes
and each paced run's p50 / p99, queue / input-wait tails, window stops and
the producer's credit wait.
usage: python tools/r05_small_window_probe.py OUT.jsonl [rounds] [window,...]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(window, out):
    if window:
        os.environ["FD_AMD_BENCH_WINDOW"] = window
    sys.path.insert(0, ROOT)
    from firedancer_amd import tango, workload
    pool = workload.sig_batch(1 << 16, 200, 77)
    sat = tango.bench_stream(0, 256, 0, *pool, 1 << 25, zero_copy=True)
    res = {"window": window or "default", "sat": round(sat["frags_per_s"] / 1e6, 2),
           "chunks": [int(sat["gpu_chunks_lat"]), int(sat["gpu_chunks_thr"])], "runs": []}
    for _ in range(3):
        for f in (0.5, 0.8):
            rate = f * sat["frags_per_s"]
            r = tango.bench_stream(0, 256, 0, *pool, int(rate * 0.5), rate=rate, zero_copy=True)
            res["runs"].append({"load": f, "p50_us": round(r["p50_ns"] / 1e3), "x": round(r["p99_ns"] / r["p50_ns"], 2),
                                "queue_p99_us": round(r["queue_p99_ns"] / 1e3), "input_p99_us": round(r["input_p99_ns"] / 1e3),
                                "stop_window": int(r["stop_window"]),
                                "credit_wait_us": round(r["producer_credit_wait_max_ns"] / 1e3),
                                "chunks": [int(r["gpu_chunks_lat"]), int(r["gpu_chunks_thr"])]})
    with open(out, "a") as f:
        f.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2], sys.argv[3])
        sys.exit(0)
    out = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    ws = sys.argv[3].split(",") if len(sys.argv) > 3 else ["", "65536"]
    for _ in range(rounds):
        for w in ws:
            rc = subprocess.call([sys.executable, os.path.abspath(__file__), "--child", w, out], timeout=300)
            if rc:
                sys.exit(rc)

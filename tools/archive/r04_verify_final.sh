#!/bin/bash
# Round 4: the -m gpu suite, the latency lines of the bench, then a zero-copy sweep of two streams through
# the tile's kernel (tools/gpu_sweep_tile.py --zero-copy).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04_verify; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu --no-stream --no-host-fed > $O/bench_latency.json 2> $O/bench_latency.err \
  || { echo "bench failed"; tail -20 $O/bench_latency.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_latency.json').read().strip().splitlines()[-1])
print(round(d['value']/1e6,2), d['latency_ms_4096']['p50'], d['latency_ms_4096_registered']['p50'], d['dropin_call_us']['p50'])"
timeout -k 10 800 python -u tools/gpu_sweep_tile.py --zero-copy 0 5 > $O/sweep_tile_zc.jsonl || { echo "sweep failed"; exit 1; }
cut -c1-300 $O/sweep_tile_zc.jsonl

#!/bin/bash
# After the FD_POOL_DBL_PCT change: gpu tests, a 2^25-signature k_dsmp sweep, default bench.
set -o pipefail
O=gpurun_out/pct100; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
FD_SWEEP_KERNEL=k_dsmp timeout -k 10 400 python -u tools/gpu_sweep.py 0 3 > $O/sweep.jsonl 2> $O/sweep.err || { echo "sweep failed"; tail -20 $O/sweep.err; cat $O/sweep.jsonl; exit 1; }
cat $O/sweep.jsonl
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['stage_ms']['k_dsm'], d.get('latency_ms_4096_registered',{}).get('p50'))"

#!/bin/bash
# HEAD re-check on one box: full -m gpu suite, a 2^25-signature parity sweep
# of the latency kernels (stream 1 forces k_dsm4, stream 2 k_dsm8), default bench.
set -o pipefail
O=gpurun_out/final_check; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 python -u tools/gpu_sweep.py 1 2 > $O/sweep.jsonl 2> $O/sweep.err || { echo "sweep failed"; tail -20 $O/sweep.err; cat $O/sweep.jsonl; exit 1; }
cat $O/sweep.jsonl
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d.get('latency_ms_4096_registered',{}).get('p50'))"

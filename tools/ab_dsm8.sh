#!/bin/bash
# k_dsm8 vs k_dsm4 on the latency path, same library: parity with k_dsm8
# forced, then interleaved k_dsm4-time scaling and bench latency rows.
set -o pipefail
mkdir -p gpurun_out
FD_AMD_DSM8=1 timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dsm8_tests.log 2>&1 || { echo "parity FAILED (k_dsm8)"; tail -30 gpurun_out/dsm8_tests.log; exit 1; }
tail -1 gpurun_out/dsm8_tests.log
for r in 1 2; do
  for v in 1 0; do
    echo "== FD_AMD_DSM8=$v"
    FD_AMD_DSM8=$v timeout -k 10 120 python3 tools/dsm4_scaling.py 2>/dev/null | python3 -c "
import json,sys
print(' '.join('%d:%.3f' % (d['n'], d['k_dsm4_ms']) for d in map(json.loads, sys.stdin)))"
    FD_AMD_DSM8=$v timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-stream --no-cpu 2>/dev/null | python3 -c "
import json,sys; d=json.load(sys.stdin); print('p50 staged %.4f registered %.4f dropin %.1f us' % (d['latency_ms_4096']['p50'], d['latency_ms_4096_registered']['p50'], d['dropin_call_us']['p50']))"
  done
done

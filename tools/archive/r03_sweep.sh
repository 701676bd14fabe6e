#!/bin/bash
# The 10^8-signature parity sweep with the HEAD kernels: streams 0-2 forced
# through the latency kernel k_dsm8 (split carry), streams 3-5 through the
# pooled k_dsmp (+ k_ai / k_fin).  usage: tools/r03_sweep.sh <tag> [streams...]
set -o pipefail
TAG=${1:-r03_sweep}; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for k in ${@:-0 1 2 3 4 5}; do
  if [ $k -lt 3 ]; then K=k_dsm8; else K=k_dsmp; fi
  FD_SWEEP_KERNEL=$K timeout -k 10 300 python3 -u tools/gpu_sweep.py $k >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "stream $k ($K) failed"; tail -20 $O/sweep.err; exit 1; }
  tail -1 $O/sweep.jsonl
done

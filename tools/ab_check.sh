#!/bin/bash
# Parity tests on the first candidate library, then interleaved A/B benches.
# usage: tools/ab_check.sh <rounds> cand.so other.so ...
set -o pipefail
R=$1; shift
mkdir -p gpurun_out
FD_AMD_LIB=$PWD/$1 timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo "parity FAILED for $1"; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
bash tools/ab_bench.sh $R "$@"

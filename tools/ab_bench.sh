#!/bin/bash
# A/B: interleaved bench runs of several library builds in one box session.
# usage: tools/ab_bench.sh <rounds> lib1.so lib2.so ...
R=$1; shift
for r in $(seq $R); do
  for lib in "$@"; do
    v=$(FD_AMD_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --steps 4 --warmup 1 --no-cpu --no-latency --no-stream 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3f Mv/s dsm %.2f ms decomp %.2f prep %.2f ok %d' % (d['value']/1e6, d['stage_ms']['k_dsm'], d['stage_ms']['k_decomp'], d['stage_ms']['k_prep'], d['verdicts']['ok']))")
    echo "$lib: $v"
  done
done

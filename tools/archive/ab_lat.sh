#!/bin/bash
# A/B of the 4096-signature latency path (k_front + k_dsm4) for several library builds.
# usage: tools/ab_lat.sh <rounds> lib1.so lib2.so ...
R=$1; shift
for r in $(seq $R); do
  for lib in "$@"; do
    v=$(FD_AMD_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-stream 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); l=d['latency_ms_4096']; print('p50 %.4f ms p99 %.4f ms  %.2f Mv/s' % (l['p50'], l['p99'], d['value']/1e6))")
    echo "$lib: $v"
  done
done

#!/bin/bash
# Interleaved A/B of the latency path: k_dsm4 time vs batch (tools/dsm4_scaling.py)
# and the registered p50 @4096 (bench latency rows), per library build.
# usage: tools/ab_lat2.sh <rounds> lib1.so lib2.so ...
R=$1; shift
for r in $(seq $R); do
  for lib in "$@"; do
    echo "== $lib"
    FD_AMD_LIB=$PWD/$lib timeout -k 10 120 python3 tools/dsm4_scaling.py 2>/dev/null | python3 -c "
import json,sys
print(' '.join('%d:%.3f' % (d['n'], d['k_dsm4_ms']) for d in map(json.loads, sys.stdin)))"
  done
done

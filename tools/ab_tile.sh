#!/bin/bash
# streaming-tile A/B of library builds: saturated rate and half-load p50 per batch_max
# usage: tools/ab_tile.sh <rounds> lib1.so lib2.so ...
export GPU_MAX_HW_QUEUES=16
R=$1; shift
for r in $(seq $R); do
  for lib in "$@"; do
    v=$(FD_AMD_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-latency 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print(' | '.join('%d: %.2f M/s p50 %.0f us' % (r['batch_max'], r['copy']['saturated_frags_per_s']/1e6, r['copy']['at_50%']['p50_us']) for r in d['stream_tile']['rows']), 'checks', d['stream_tile']['all_checks_pass'])") || exit 1
    echo "$lib: $v"
  done
done

#!/bin/bash
# Interleaved A/B of the tile bench's CPU choice (FD_AMD_BENCH_CPU_PICK=top: the round-4 rule, the
# highest-numbered CPUs; default: the quietest CPUs, one per core): the stream_tile rows of bench.py.
#   tools/r05_ab_cpupick.sh OUTDIR [ROUNDS]
o=$1; rounds=${2:-2}; mkdir -p $o
for i in $(seq 1 $rounds); do
  for V in top quiet; do
    FD_AMD_BENCH_CPU_PICK=$V timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu --no-latency --no-host-fed \
      --detail $o/detail_${V}_$i.json > $o/line_${V}_$i.json 2> $o/err_${V}_$i.txt || exit 1
    grep "spinning threads" $o/err_${V}_$i.txt | head -1
    python3 -c "
import json; d=json.load(open('$o/line_${V}_$i.json'))['stream_tile']
print('$V $i', d['every_row_worst_p99_within_2_5x_p50'], [(r['bmax'], r['mode'][0], round(r['sat']/1e6,1), r['worst_x_50'], r['worst_x_80']) for r in d['rows']], 'fixed', d['fixed_1M_4096'])"
  done
done

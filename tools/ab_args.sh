#!/bin/bash
# bench A/B of command-line variants on one library build
# usage: tools/ab_args.sh <rounds> "<args A>" "<args B>" ...
export GPU_MAX_HW_QUEUES=16
R=$1; shift
for r in $(seq $R); do
  for a in "$@"; do
    v=$(timeout -k 10 200 python3 bench.py --steps 12 --warmup 2 --no-cpu --no-latency --no-stream $a 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3f Mv/s  %.3f ms/step  dsm %.2f ms  frac %.3f ok %d' % (d['value']/1e6, d['ms_per_step'], d['stage_ms']['k_dsm'], d['roofline']['frac'], d['verdicts']['ok']))") || exit 1
    echo "[$a]: $v"
  done
done

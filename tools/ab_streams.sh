#!/bin/bash
# bench A/B: throughput DSM kernel x streams in flight, interleaved rounds
# usage: tools/ab_streams.sh <rounds> "<kernel:streams> ..."
export GPU_MAX_HW_QUEUES=16
R=${1:-2}; CASES=${2:-"k_dsm:1 k_dsm:2 k_dsmp:1 k_dsmp:2"}
for r in $(seq $R); do
  for c in $CASES; do
    k=${c%%:*}; ns=${c##*:}
    v=$(timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --no-cpu --no-latency --no-stream --streams $ns --dsm-kernel $k 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3f Mv/s  %.3f ms/step  dsm %.2f ms  frac %.3f ok %d' % (d['value']/1e6, d['ms_per_step'], d['stage_ms']['k_dsm'], d['roofline']['frac'], d['verdicts']['ok']))") || exit 1
    echo "$k streams=$ns: $v"
  done
done

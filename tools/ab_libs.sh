#!/bin/bash
# bench A/B of library builds on a fixed DSM kernel and stream count
# usage: tools/ab_libs.sh <rounds> <kernel> <streams> lib1.so lib2.so ...
export GPU_MAX_HW_QUEUES=16
R=$1; K=$2; NS=$3; shift 3
for r in $(seq $R); do
  for lib in "$@"; do
    v=$(FD_AMD_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --no-cpu --no-latency --no-stream --streams $NS --dsm-kernel $K 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3f Mv/s  %.3f ms/step  dsm %.2f ms  frac %.3f ok %d' % (d['value']/1e6, d['ms_per_step'], d['stage_ms']['k_dsm'], d['roofline']['frac'], d['verdicts']['ok']))") || exit 1
    echo "$lib: $v"
  done
done

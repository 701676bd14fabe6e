#!/bin/bash
# k_dsmp scheduling constants A/B (interleaved, one box): ab/pool_p0.so default
# (FD_POOL_DBL_PCT 78, FD_POOL_REFILL 8), p1 DBL_PCT 70, p2 86, p3 REFILL 4, p4 16, p5 DBL_PCT 92, p6 100.
set -o pipefail
O=gpurun_out/pooltune; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for lib in ${LIBS:-ab/pool_p0.so ab/pool_p2.so ab/pool_p5.so ab/pool_p6.so}; do
    v=$(FD_AMD_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --no-cpu --no-latency --no-stream --no-host-fed 2>>$O/ab.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3f Mv/s  %.3f ms/step  dsm %.3f ms  frac %.4f ok %d' % (d['value']/1e6, d['ms_per_step'], d['stage_ms']['k_dsm'], d['roofline']['frac'], d['verdicts']['ok']))") || { echo "ab failed $lib"; tail -20 $O/ab.err; exit 1; }
    echo "$lib: $v" | tee -a $O/ab.txt
  done
done

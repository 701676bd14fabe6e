#!/bin/bash
# One box session: k_dsmp A/B of library variants (interleaved), then the
# persistent-tile check (tests + probes).  usage: tools/r03_session.sh <tag> lib...
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for lib in "$@"; do
    v=$(FD_AMD_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --no-cpu --no-latency --no-stream --no-host-fed --streams 1 2>>$O/ab.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3f Mv/s  %.3f ms/step  dsm %.3f ms  frac %.4f ok %d' % (d['value']/1e6, d['ms_per_step'], d['stage_ms']['k_dsm'], d['roofline']['frac'], d['verdicts']['ok']))") || { echo "ab failed $lib"; tail -20 $O/ab.err; exit 1; }
    echo "$lib: $v" | tee -a $O/ab.txt
  done
done
bash tools/r03_tile_check.sh $TAG/tile

#!/bin/bash
# Tile A/B: host-side per-frag divisions (frame % frame_cnt, bench producer/consumer seq % n)
set -o pipefail
O=gpurun_out/tdiv; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_tile_gpu.py tests/test_tile_cut.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tile tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for lib in ab/tdiv0.so ab/tdiv1.so; do
    for a in "16384 2097152 zc check" "4096 1048576 zc check" "16384 2097152 check"; do
      FD_AMD_LIB=$PWD/$lib timeout -k 10 120 python -u tools/tile_probe.py $a > $O/p.json 2>&1 || { echo "probe failed $lib $a"; cat $O/p.json; exit 1; }
      python3 -c "
import json,sys
rows=[json.loads(l) for l in open('$O/p.json') if l.startswith('{')]
print('$lib', '$a', ' | '.join('%.2fM p50 %.2f p99 %.2f ms mism %d' % (r['frags_per_s']/1e6, r['p50_ns']/1e6, r['p99_ns']/1e6, r['mismatches']) for r in rows))
" | tee -a $O/ab.txt
    done
  done
done

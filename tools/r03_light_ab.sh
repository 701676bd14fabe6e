#!/bin/bash
# Tile latency-mode threshold A/B (FD_AMD_TILE_LIGHT_FRAGS: default 32 x CUs = 8192), saturated and half load.
set -o pipefail
O=gpurun_out/light; mkdir -p $O
for r in 1 2; do
  for L in 8192 16384 32768; do
    for a in "4096 1048576 check" "16384 2097152 check" "16384 2097152 zc check"; do
      FD_AMD_TILE_LIGHT_FRAGS=$L timeout -k 10 120 python -u tools/tile_probe.py $a > $O/p.json 2>&1 || { echo "probe failed $L $a"; cat $O/p.json; exit 1; }
      python3 -c "
import json
rows=[json.loads(l) for l in open('$O/p.json') if l.startswith('{')]
print('light $L', '$a', ' | '.join('%.2fM p50 %.2f p99 %.2f ms mism %d' % (r['frags_per_s']/1e6, r['p50_ns']/1e6, r['p99_ns']/1e6, r['mismatches']) for r in rows))
" | tee -a $O/ab.txt
    done
  done
done

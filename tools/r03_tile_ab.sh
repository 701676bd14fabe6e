#!/bin/bash
# Persistent tile A/B probes (saturated + half load, zero-copy, checked).
# usage: tools/r03_tile_ab.sh <tag> <frags> "<ENV=..>" ["<ENV=..>" ...]
set -o pipefail
TAG=$1; NF=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
for cfg in "$@"; do
  for b in ${BMAXES:-256 16384}; do
    echo "== $cfg bmax $b" >> $O/ab.txt
    env $cfg FD_AMD_TILE_DEBUG=1 timeout -k 10 120 python3 -u tools/tile_probe.py $b $NF ${MODE-zc} check >> $O/ab.txt 2>&1 || { echo "probe failed: $cfg $b"; tail -20 $O/ab.txt; exit 1; }
  done
done
cat $O/ab.txt

#!/bin/bash
# Interleaved A/B of the resident headline's batches in flight (bench.py --streams):
#   tools/r05_ab_streams.sh OUT "3 4" [ROUNDS]
out=$1; ss=$2; rounds=${3:-3}
for i in $(seq 1 $rounds); do
  for S in $ss; do
    echo "== streams $S round $i" >> $out
    timeout -k 10 120 python bench.py --steps 30 --warmup 5 --streams $S --no-stream --no-cpu --no-latency --no-host-fed \
      --detail /tmp/d.json >> $out 2>&1 || exit 1
  done
done

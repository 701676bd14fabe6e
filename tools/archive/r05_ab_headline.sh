#!/bin/bash
# Interleaved A/B of the resident headline (bench.py configs[1] line only):
#   tools/r05_ab_headline.sh OUT LIB_A LIB_B [ROUNDS]
# LIB_* : "" for the product library, else a path to an A/B build.
out=$1; a=$2; b=$3; rounds=${4:-3}
for i in $(seq 1 $rounds); do
  for L in "$a" "$b"; do
    if [ -n "$L" ]; then export FD_AMD_LIB=$PWD/$L; else unset FD_AMD_LIB; fi
    echo "== ${L:-product} round $i" >> $out
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-stream --no-cpu --no-latency --no-host-fed \
      --detail /tmp/d.json >> $out 2>&1 || exit 1
  done
done

#!/bin/bash
# Interleaved A/B of the HIP hardware queues behind the resident headline's
# streams: GPU_MAX_HW_QUEUES unset (the runtime's 4, of which the bench's four
# streams get two) vs the values given, each at the given --streams.
#   tools/r05_ab_hwq.sh OUT "8 16" "4 6" [ROUNDS]
out=$1; qs=$2; ss=$3; rounds=${4:-3}
for i in $(seq 1 $rounds); do
  for S in $ss; do
    for Q in default $qs; do
      echo "== hwq $Q streams $S round $i" >> $out
      if [ "$Q" = default ]; then
        timeout -k 10 120 python bench.py --steps 30 --warmup 5 --streams $S --no-stream --no-cpu --no-latency \
          --no-host-fed --detail /tmp/d.json >> $out 2>&1 || exit 1
      else
        GPU_MAX_HW_QUEUES=$Q timeout -k 10 120 python bench.py --steps 30 --warmup 5 --streams $S --no-stream --no-cpu \
          --no-latency --no-host-fed --detail /tmp/d.json >> $out 2>&1 || exit 1
      fi
    done
  done
done

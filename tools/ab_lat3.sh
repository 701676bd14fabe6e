#!/bin/bash
# latency A/B of library builds: GPU-only stage times at 4096 (tools/lat_floor.py) and the bench's
# p50 rows (registered, staged, drop-in).  usage: tools/ab_lat3.sh <rounds> lib1.so lib2.so ...
# HIP default hardware queues
R=$1; shift
for r in $(seq $R); do
  for lib in "$@"; do
    f=$(FD_AMD_LIB=$PWD/$lib timeout -k 10 120 python3 tools/lat_floor.py 2>/dev/null | grep "^4096 " | cut -d' ' -f2-) || exit 1
    b=$(FD_AMD_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-stream 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('p50 reg %.4f staged %.4f dropin %.1f us' % (d['latency_ms_4096_registered']['p50'], d['latency_ms_4096']['p50'], d['dropin_call_us']['p50']))") || exit 1
    echo "$lib: $f | $b"
  done
done

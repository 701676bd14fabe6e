#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_lat; mkdir -p $O
timeout -k 10 400 python3 tools/r05_latency_ab.py $O/lat_ab.jsonl ",build_ab/lib_front_prepfirst.so" 3 300 > $O/lat_ab.log 2>&1 || { echo "lat ab failed"; tail -20 $O/lat_ab.log; exit 1; }
echo "lat ok"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace3 -o run -- python3 bench.py --steps 8 --warmup 3 \
  --no-cpu --no-latency --no-stream --no-host-fed > $O/trace3.log 2>&1 || { echo "trace failed"; tail -20 $O/trace3.log; exit 1; }
echo "trace ok"

#!/bin/bash
# Round-4 measurement set on one GPU box (each step time-limited, chained): the default bench line
# (headline, stream_tile rows, TXN row, CPU baseline), rocprof kernel stats and PMC passes of the
# headline kernels, the config-4 transaction bench.
# usage: tools/r04_final_measure.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r04_final}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 1 \
  --streams 1 --no-cpu --no-latency --no-stream --no-host-fed > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
echo "rocprof ok"
bash tools/prof_pmc.sh $O/pmc > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
echo "pmc ok"
timeout -k 10 300 python3 bench.py --workload txn --steps 5 --warmup 1 > $O/txn.json 2> $O/txn.err || { echo "txn bench failed"; tail -20 $O/txn.err; exit 1; }
echo "txn ok"

#!/bin/bash
# Persistent verify tile on the GPU box: one tile test first (bounded), the
# tile test file, then saturated + half-load probes at batch_max 256 / 4096 /
# 16384, zero-copy and copy, with every frag checked (bytes of every 16th).
# usage: tools/r03_tile_check.sh <tag> [probe frags]
set -o pipefail
TAG=${1:-tile}; NF=${2:-2000000}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python3 -u -m pytest "tests/test_tile_gpu.py::test_tile_publishes_passing_frags_in_order[512-4096-False]" -x -v --timeout 90 --timeout-method thread > $O/first.log 2>&1 || { echo "first tile test failed"; tail -40 $O/first.log; exit 1; }
tail -3 $O/first.log
timeout -k 10 400 python3 -u -m pytest tests/test_tile_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tile tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 -u -m pytest tests/test_engine_api_gpu.py -x -v --timeout 120 --timeout-method thread > $O/api.log 2>&1 || { echo "engine api tests failed"; tail -40 $O/api.log; exit 1; }
tail -3 $O/api.log
for b in 256 4096 16384; do
  for m in zc ""; do
    timeout -k 10 120 python3 -u tools/tile_probe.py $b $NF $m check >> $O/probe.jsonl 2>> $O/probe.err || { echo "probe $b $m failed"; tail -20 $O/probe.err; exit 1; }
  done
done
cat $O/probe.jsonl

#!/bin/bash
# Kernel trace of the streaming tile (batch path) at one batch_max:
# saturated then 50 % load, zero copy, every frag checked.
# usage: tools/r03_tile_trace.sh <tag> <batch_max> [frags]
set -o pipefail
O=gpurun_out/$1; B=${2:-16384}; NF=${3:-1000000}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/tile_probe.py $B $NF zc check > $O/probe.jsonl 2> $O/probe.err || { echo "trace failed"; tail -20 $O/probe.err; exit 1; }
cat $O/probe.jsonl | cut -c1-300
find $O/trace -name "*kernel_stats.csv" -exec cat {} \;

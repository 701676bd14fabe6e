#!/bin/bash
# config 4 at 2^24 with every transaction re-checked by the reference; tile knob A/B at 16384.
set -o pipefail
O=gpurun_out/r03_s3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u bench.py --workload txn --steps 5 --warmup 1 --txn-full-check > $O/txn_full.json 2> $O/txn_full.err || { echo "txn full check failed"; tail -20 $O/txn_full.err; exit 1; }
cut -c1-300 $O/txn_full.json; python3 -c "import json; d=json.load(open('$O/txn_full.json')); print(d['verdicts'])"
BMAXES="16384" bash tools/r03_tile_ab.sh r03_s3/tile 1000000 "X=0" "FD_AMD_TILE_LIGHT_FRAGS=2048" "FD_AMD_TILE_WINDOW=524288" "FD_AMD_TILE_WINDOW=131072" "FD_AMD_TILE_CHUNK_WAIT_NS=200000" > /dev/null || exit 1
grep -E "^==|tile debug|frags_per_s" $O/tile/ab.txt | cut -c1-200

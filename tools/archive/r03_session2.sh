#!/bin/bash
# GPU tests, latency A/B of two builds, multi-GPU rehearsals.
set -o pipefail
O=gpurun_out/r03_s2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_lat3.sh 2 ab/lat0.so ab/lat1.so > $O/lat_ab.txt 2>&1 || { echo "lat ab failed"; cat $O/lat_ab.txt; exit 1; }
cat $O/lat_ab.txt
bash tools/r03_multi.sh r03_s2/multi || exit 1

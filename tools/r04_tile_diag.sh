#!/bin/bash
# Round 4 tile stall hunt, kernel side: no initial scout clock store; no claim stamp / res_time
# store; profiling flag at run time; everything reverted (sanity).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
K="publishes_passing_frags_in_order or stream_bench_smoke"
for v in allrev vgpr248 noinit norestime profrt; do
  FD_AMD_LIB=$PWD/ab/$v.so timeout -k 10 200 python -u -m pytest tests/test_tile_gpu.py -k "$K" -v -s --durations=0 \
    --timeout 60 --timeout-method thread > gpurun_out/r04_diag_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc passed=$(grep -c PASSED gpurun_out/r04_diag_$v.log)"; grep -E "FAILED|fd_verify_amd_tile_run:" gpurun_out/r04_diag_$v.log | head -3
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done

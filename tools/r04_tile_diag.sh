#!/bin/bash
# Round 4: host-side A/B of the tile run loop (plain-store heartbeat; no periodic hipEventQuery;
# publisher inline; all three) on the first tile tests; then, with the first variant that passes,
# the whole tile test file and the streaming rows of the bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
K="publishes_passing_frags_in_order or stream_bench_smoke"
good=""
for v in product noquery beatst pubinl; do
  lib=$PWD/ab/$v.so; [ $v = product ] && lib=$PWD/firedancer_amd/libfd_ed25519_amd.so
  FD_AMD_LIB=$lib timeout -k 10 200 python -u -m pytest tests/test_tile_gpu.py -k "$K" -v -s --timeout 60 \
    --timeout-method thread > gpurun_out/r04_diag_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc passed=$(grep -c PASSED gpurun_out/r04_diag_$v.log)"; grep -E "FAILED|fd_verify_amd_tile_run:" gpurun_out/r04_diag_$v.log | head -4
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  if [ $rc -eq 0 ] && [ -z "$good" ]; then good=$v; fi
done
echo "first passing variant: ${good:-none}"
[ -z "$good" ] && exit 0
glib=$PWD/ab/$good.so; [ $good = product ] && glib=$PWD/firedancer_amd/libfd_ed25519_amd.so
FD_AMD_LIB=$glib timeout -k 10 500 python -u -m pytest tests/test_tile_gpu.py -v --timeout 120 \
  --timeout-method thread > gpurun_out/r04_tile_tests_$good.log 2>&1
echo "full tile tests ($good) rc=$?"; grep -E "FAILED|passed|failed" gpurun_out/r04_tile_tests_$good.log | tail -8
FD_AMD_LIB=$glib timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-latency --no-host-fed \
  --stream-frags 1048576 > gpurun_out/r04_bench_tile_$good.json 2> gpurun_out/r04_bench_tile_$good.err
echo "bench rc=$?"; tail -2 gpurun_out/r04_bench_tile_$good.err

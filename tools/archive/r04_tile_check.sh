#!/bin/bash
# Round 4: the tile GPU tests, then the streaming rows of the bench (no CPU baseline / latency / host-fed legs).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_tile_gpu.py -v --durations=0 --timeout 120 --timeout-method thread \
  > gpurun_out/r04_tile_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|fd_verify_amd_tile_run:" gpurun_out/r04_tile_tests.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-latency --no-host-fed --stream-frags 4194304 \
  > gpurun_out/r04_bench_tile.json 2> gpurun_out/r04_bench_tile.err
rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/r04_bench_tile.err
exit $rc

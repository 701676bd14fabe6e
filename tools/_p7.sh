mkdir -p gpurun_out/p7
export FD_AMD_TILE_PROF=1
D=$PWD/firedancer_amd/libfd_ed25519_amd_diag.so
FD_AMD_LIB=$D FD_AMD_TILE_POOL=1 timeout -k 10 200 python -u tools/tile_probe.py 16384 4194304 zc > gpurun_out/p7/pool.log 2>&1 || exit 1
FD_AMD_TILE_POOL=1 timeout -k 10 300 python -u -m pytest tests/test_tile_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p7/tiles_pool.log 2>&1; echo pool-tests=$?
cut -c1-1200 gpurun_out/p7/pool.log; tail -n 3 gpurun_out/p7/tiles_pool.log

#!/bin/bash
# Round 4: the whole -m gpu suite, then the 2-rank torchrun rehearsal of the N-GPU bench on a one-GPU
# box (FD_AMD_DEVICE_MAP=mod maps both ranks onto device 0; each rank's tile gets half the wave slots):
# the headline line with host_fed_node and stream_tile_node (per-rank tile rows and node sums).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r04_rehearsal}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
FD_AMD_DEVICE_MAP=mod timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29521 bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu > $O/bench_2rank.json 2> $O/bench_2rank.err \
  || { echo "2-rank bench failed"; tail -20 $O/bench_2rank.err; exit 1; }
echo "2-rank ok"
cut -c1-600 $O/bench_2rank.json

#!/bin/bash
# Multi-GPU rehearsal on a one-GPU box (ranks / engines mapped onto device 0
# with FD_AMD_DEVICE_MAP=mod): 2-rank bench with the host-fed node rate,
# 2-rank txn bench, native multi-engine from one process.
set -o pipefail
O=gpurun_out/${1:-r03_multi}; mkdir -p $O
export TMPDIR=/tmp
FD_AMD_DEVICE_MAP=mod timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu > $O/bench_2rank.json 2> $O/bench_2rank.err || { echo "2-rank bench failed"; tail -20 $O/bench_2rank.err; exit 1; }
echo "2-rank ok"
FD_AMD_DEVICE_MAP=mod timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --workload txn --total-sigs 4194304 --steps 3 --warmup 1 > $O/txn_2rank.json 2> $O/txn_2rank.err || { echo "2-rank txn failed"; tail -20 $O/txn_2rank.err; exit 1; }
echo "2-rank txn ok"
FD_AMD_DEVICE_MAP=mod timeout -k 10 300 python3 bench.py --multi-engine --gpus 2 --steps 4 --warmup 1 > $O/multi_engine_2.json 2> $O/multi_engine_2.err || { echo "multi-engine failed"; tail -20 $O/multi_engine_2.err; exit 1; }
echo "multi-engine ok"
cat $O/bench_2rank.json $O/txn_2rank.json $O/multi_engine_2.json | cut -c1-1500

#!/bin/bash
# Round-end measurement set on one GPU box (each step time-limited, chained):
# bench line, rocprof kernel stats, PMC passes, config-4 txn bench, and the
# 2-rank torchrun rehearsal (ranks mapped onto device 0).
# usage: tools/final_measure.sh <tag>
set -o pipefail
T=${1:-final}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 1 --streams 1 --no-cpu --no-latency --no-stream --no-host-fed > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
echo "rocprof ok"
bash tools/prof_pmc.sh $O/pmc > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
echo "pmc ok"
timeout -k 10 300 python3 bench.py --workload txn --steps 5 --warmup 1 > $O/txn.json 2> $O/txn.err || { echo "txn bench failed"; tail -20 $O/txn.err; exit 1; }
echo "txn ok"
FD_AMD_DEVICE_MAP=mod timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 4 --warmup 1 > $O/bench_2rank.json 2> $O/bench_2rank.err || { echo "2-rank bench failed"; tail -20 $O/bench_2rank.err; exit 1; }
FD_AMD_DEVICE_MAP=mod timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --workload txn --total-sigs 4194304 --steps 3 --warmup 1 > $O/txn_2rank.json 2> $O/txn_2rank.err || { echo "2-rank txn failed"; tail -20 $O/txn_2rank.err; exit 1; }
echo "2-rank ok"
FD_AMD_DEVICE_MAP=mod timeout -k 10 300 python3 bench.py --multi-engine --gpus 2 --steps 4 --warmup 1 > $O/multi_engine_2.json 2> $O/multi_engine_2.err || { echo "multi-engine failed"; tail -20 $O/multi_engine_2.err; exit 1; }
echo "multi-engine ok"

#!/bin/bash
# Round-end measurement set on one GPU box (each step time-limited, chained with
# exits; run as separate gpurun calls by stage so each stays within a call's limit):
#   bench    the driver's default bench line (+ detail), the GPU suite first
#   prof     rocprofv3 --stats of the headline kernels and their PMC passes (the files the bench
#            line's frac_rocprof / held_clock_ghz / traffic read: profiles/rNN_rocprof_kernel_stats.csv,
#            profiles/rNN_pmc_latest.json), then the tile kernel's stats + PMC (tools/prof_tile.sh)
#   multi    the config-4 txn bench and the 2-rank rehearsals (ranks mapped onto device 0)
#   sweep    the >= 10^8 parity sweep of the headline kernels (every hot-kernel change ends here:
#            six 2^24 streams through k_dsmp at 2^20 batches, two through k_dsm8) -- two calls:
#            `sweep a` streams 0-3, `sweep b` streams 4-5 + the k_dsm8 pair
#   tilesweep  the same streams through k_tile_persist, every chunk level (quad included)
# usage: tools/final_measure.sh <tag> bench|prof|multi|sweep a|sweep b|tilesweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-final}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
case "$2" in
bench)
  timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -20 $O/gpu_tests.log; exit 1; }
  echo "gpu tests ok"
  timeout -k 10 600 python3 bench.py --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
  echo "bench ok" ;;
prof)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 1 \
    --streams 1 --no-cpu --no-latency --no-stream --no-host-fed > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
  echo "rocprof ok"
  bash tools/prof_pmc.sh $O/pmc > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
  python3 tools/pmc_summary.py $O/pmc 1048576 > $O/pmc_summary.json || { echo "pmc summary failed"; exit 1; }
  echo "pmc ok"
  timeout -k 10 600 bash tools/prof_tile.sh $T/prof_tile 4194304 > $O/prof_tile.log 2>&1 || { echo "tile prof failed"; tail -20 $O/prof_tile.log; exit 1; }
  echo "tile prof ok" ;;
multi)
  timeout -k 10 300 python3 bench.py --workload txn --steps 5 --warmup 1 --detail $O/txn_detail.json > $O/txn.json 2> $O/txn.err || { echo "txn bench failed"; tail -20 $O/txn.err; exit 1; }
  echo "txn ok"
  FD_AMD_DEVICE_MAP=mod timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 > $O/bench_2rank.json 2> $O/bench_2rank.err || { echo "2-rank bench failed"; tail -20 $O/bench_2rank.err; exit 1; }
  echo "2-rank ok"
  FD_AMD_DEVICE_MAP=mod timeout -k 10 300 python3 bench.py --multi-engine --gpus 2 --steps 4 --warmup 1 > $O/multi_engine_2.json 2> $O/multi_engine_2.err || { echo "multi-engine failed"; tail -20 $O/multi_engine_2.err; exit 1; }
  echo "multi-engine ok" ;;
sweep)
  if [ "$3" = "a" ]; then S="0:k_dsmp 1:k_dsmp 2:k_dsmp 3:k_dsmp"; else S="4:k_dsmp 5:k_dsmp 0:k_dsm8 1:k_dsm8"; fi
  timeout -k 10 1000 python3 -u tools/gpu_sweep.py $S > $O/sweep_$3.jsonl 2> $O/sweep_$3.err || { echo "sweep failed"; tail -5 $O/sweep_$3.err; exit 1; }
  echo "sweep ok" ;;
tilesweep)
  timeout -k 10 1000 python3 -u tools/gpu_sweep_tile.py --zero-copy 0 1 > $O/tilesweep_zc.jsonl 2> $O/tilesweep_zc.err || { echo "tile sweep failed"; tail -5 $O/tilesweep_zc.err; exit 1; }
  echo "tile sweep ok" ;;
*) echo "usage: tools/final_measure.sh <tag> bench|prof|multi|sweep a|sweep b|tilesweep"; exit 2 ;;
esac

#!/bin/bash
# per-lane k_dsm A/B: resident throughput with k_dsm forced (one stream) and the registered host path
# (2^17-signature chunks, which take k_dsm).  usage: tools/ab_dsm_host.sh <rounds> lib1.so lib2.so ...
export GPU_MAX_HW_QUEUES=16
R=$1; shift
for r in $(seq $R); do
  for lib in "$@"; do
    v=$(FD_AMD_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --steps 6 --warmup 1 --no-cpu --no-stream --streams 1 --dsm-kernel k_dsm 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('k_dsm %.2f Mv/s stage %.2f ms | host reg %.2f staged %.2f Mv/s' % (d['value']/1e6, d['stage_ms']['k_dsm'], d['host_soa_registered']['verifies_per_s']/1e6, d['host_soa']['verifies_per_s']/1e6))") || exit 1
    echo "$lib: $v"
  done
done

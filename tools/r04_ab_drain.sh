#!/bin/bash
# Round 4 A/B: k_dsmp drain priority (FD_POOL_DRAIN_PRIO 0 / 1), interleaved, headline bench without the
# CPU, latency, host-fed and stream rows; then the latency-path A/B (diagnostics library).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04_ab_drain; mkdir -p $O
for r in 1 2 3; do
  for v in 0 1; do
    FD_AMD_LIB=firedancer_amd/libfd_ab_drainprio$v.so timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 \
      --no-cpu --no-latency --no-host-fed --no-stream > $O/prio${v}_$r.json 2> $O/prio${v}_$r.err \
      || { echo "bench prio$v run $r failed"; tail -20 $O/prio${v}_$r.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('$O/prio${v}_$r.json').read().strip().splitlines()[-1])
print('prio$v run $r', round(d['value']/1e6,2), d.get('stage_ms'), d['roofline'].get('frac'))"
  done
done
timeout -k 10 200 python3 tools/latency_ab.py 4096 400 > $O/latency_ab_4096.jsonl && \
timeout -k 10 200 python3 tools/latency_ab.py 1024 400 > $O/latency_ab_1024.jsonl && cat $O/latency_ab_*.jsonl

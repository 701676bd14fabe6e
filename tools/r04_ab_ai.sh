#!/bin/bash
# Round 4 A/B: k_ai at 2 / 3 waves per SIMD (FD_AI_WAVES), interleaved: headline bench without the
# CPU, latency, host-fed and stream rows (stage_ms k_dsm = k_ai + k_dsmp + k_fin alone on one stream).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04_ab_ai; mkdir -p $O
for r in 1 2 3; do
  for v in 2 3; do
    FD_AMD_LIB=firedancer_amd/libfd_ab_ai$v.so timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 \
      --no-cpu --no-latency --no-host-fed --no-stream > $O/ai${v}_$r.json 2> $O/ai${v}_$r.err \
      || { echo "bench ai$v run $r failed"; tail -20 $O/ai${v}_$r.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('$O/ai${v}_$r.json').read().strip().splitlines()[-1])
print('ai$v run $r', round(d['value']/1e6,2), d.get('stage_ms'), d['roofline'].get('frac'))"
  done
done

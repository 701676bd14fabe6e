#!/bin/bash
# Round 4: k_ai kernel time under rocprof (tools/kai_probe.py, one resident 2^20 batch, k_dsmp forced),
# with the library given as $1 (default: the product library), twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04_kai; mkdir -p $O
export TMPDIR=/tmp
L=${1:-firedancer_amd/libfd_ed25519_amd.so}
for v in a b; do
  FD_AMD_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 tools/kai_probe.py \
    > $O/$v.log 2>&1 || { echo "$v failed"; tail -20 $O/$v.log; exit 1; }
  python3 -c "
import csv,glob
for f in glob.glob('$O/$v/**/run_kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if r['Name'].split('(')[0] in ('k_ai','k_dsmp','k_fin','k_decomp','k_prep'): print('$v', r['Name'].split('(')[0], r['Calls'], round(float(r['AverageNs'])/1e6,3))"
done

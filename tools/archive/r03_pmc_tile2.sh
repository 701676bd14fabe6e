#!/bin/bash
# Memory-side counters of the persistent tile kernel: throughput chunks only
# (FD_AMD_TILE_LIGHT_FRAGS=0) vs latency chunks only, plus the batch kernels.
set -o pipefail
O=gpurun_out/${1:-r03_pmc_tile2}
mkdir -p $O
export TMPDIR=/tmp
P1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"
P2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
P3="SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_FLAT"
k=0
for lf in 0 1000000000; do
  for P in "$P1" "$P2" "$P3"; do
    k=$((k+1))
    FD_AMD_TILE_LIGHT_FRAGS=$lf timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$k -o run -- python3 tools/pmc_tile.py $([ $lf = 0 ] && echo both || echo tile) > $O/p$k.log 2>&1 || { echo "pmc pass $k failed"; tail -20 $O/p$k.log; exit 1; }
    f=$(find $O/p$k -name "*counter_collection.csv" | head -1)
    python3 - "$f" "$lf" >> $O/summary.txt <<'PY'
import csv,collections,sys
rows=list(csv.DictReader(open(sys.argv[1])))
agg=collections.defaultdict(float)
for r in rows:
    agg[(r['Kernel_Name'][:24], r['Counter_Name'])]+=float(r['Counter_Value'])
for k,v in sorted(agg.items()):
    if k[0].startswith(('k_tile','k_dsm','k_prep','k_decomp')): print('lf=%-10s %-26s %-34s %.4g'%(sys.argv[2],k[0],k[1],v))
PY
  done
done
cat $O/summary.txt

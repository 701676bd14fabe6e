#!/bin/bash
# Where the persistent tile kernel's waves stall: L2 request classes and tag
# stalls, SQ wait/active split, TA/TD busy; tile run (zero copy, 16384) and
# the batch kernels for comparison (tools/pmc_tile.py both).
set -o pipefail
O=gpurun_out/${1:-r03_pmc_tile3}
mkdir -p $O
export TMPDIR=/tmp
P1="TCC_UC_REQ_sum TCC_NC_REQ_sum TCC_TAG_STALL_sum TCC_BUSY_sum"
P2="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_SCA"
P3="TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum"
k=0
for P in "$P1" "$P2" "$P3"; do
  k=$((k+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$k -o run -- python3 tools/pmc_tile.py both > $O/p$k.log 2>&1 || { echo "pmc pass $k failed"; tail -20 $O/p$k.log; exit 1; }
  f=$(find $O/p$k -name "*counter_collection.csv" | head -1)
  python3 - "$f" >> $O/summary.txt <<'PY'
import csv,collections,sys
rows=list(csv.DictReader(open(sys.argv[1])))
agg=collections.defaultdict(float)
for r in rows:
    agg[(r['Kernel_Name'][:24], r['Counter_Name'])]+=float(r['Counter_Value'])
for k,v in sorted(agg.items()):
    if k[0].startswith(('k_tile','k_dsm','k_prep','k_decomp')): print('%-26s %-34s %.4g'%(k[0],k[1],v))
PY
done
cat $O/summary.txt

#!/bin/bash
# I-cache / issue counters of the persistent tile kernel vs the batch kernels.
set -o pipefail
O=gpurun_out/${1:-r03_pmc_tile}
mkdir -p $O
export TMPDIR=/tmp
export FD_AMD_TILE_LIGHT=0
timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/p1 -o run -- python3 tools/pmc_tile.py both > $O/p1.log 2>&1 || { echo "pmc pass failed"; tail -30 $O/p1.log; exit 1; }
find $O/p1 -name "*counter_collection.csv" | head -1 | xargs -I{} python3 -c "
import csv,collections,sys
rows=list(csv.DictReader(open('{}')))
agg=collections.defaultdict(float)
for r in rows:
    agg[(r['Kernel_Name'][:40], r['Counter_Name'])]+=float(r['Counter_Value'])
for k,v in sorted(agg.items()): print('%-42s %-22s %.4g'%(k[0],k[1],v))
" > $O/summary.txt
cat $O/summary.txt

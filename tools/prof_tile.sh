#!/bin/bash
# rocprofv3 kernel stats and PMC passes of the persistent tile kernel (k_tile_persist) on one saturated
# batch_max-16384 zero-copy run (tools/pmc_tile.py tile, FRAGS frags, default 2^22).  One pass per counter
# group (gfx950 limits: 8 SQ, 4 TCC with FETCH_SIZE = 3 / WRITE_SIZE = 2, 2 GRBM).  Summary per frag
# (VALU instructions, issue busy, HBM bytes, LDS conflicts) in <out>/summary.txt.
# usage: tools/prof_tile.sh <out name> [frags]   (round 4: r04_prof_tile, 2^20 frags)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-prof_tile}
F=${2:-4194304}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 tools/pmc_tile.py tile $F \
  > $O/stats.log 2>&1 || { echo "stats pass failed"; tail -20 $O/stats.log; exit 1; }
run() { name=$1; shift; timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o run -- python3 tools/pmc_tile.py tile $F \
  > $O/$name.log 2>&1 || { echo "pass $name failed"; tail -20 $O/$name.log; exit 1; }; }
run sq1  SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run sq2  SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS
run fetch FETCH_SIZE
run write WRITE_SIZE
run grbm GRBM_GUI_ACTIVE GRBM_COUNT
python3 - $O $F > $O/summary.txt <<'PY'
import csv, collections, glob, sys
O, F = sys.argv[1], float(sys.argv[2])
agg = collections.defaultdict(float)
for f in glob.glob(O + "/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_tile_persist" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    print("k_tile_persist %-22s %.6g   per frag %.6g" % (k, v, v / F))
if agg.get("GRBM_GUI_ACTIVE") and agg.get("SQ_INSTS_VALU"):
    cyc = agg["GRBM_GUI_ACTIVE"] / 8.0                       # per XCD
    print("VALU issue busy (4 cycles per wave64 instruction, 1024 SIMDs): %.3f" % (4.0 * agg["SQ_INSTS_VALU"] / 1024.0 / cyc))
    print("VALU issue busy (4.13 cycles, the per-opcode mix of s6):        %.3f" % (4.13 * agg["SQ_INSTS_VALU"] / 1024.0 / cyc))
if agg.get("FETCH_SIZE") is not None and agg.get("WRITE_SIZE") is not None:
    print("HBM bytes per frag, 2 x FETCH + WRITE (KB x 1024): %.0f; raw FETCH + WRITE: %.0f"
          % ((2 * agg["FETCH_SIZE"] + agg["WRITE_SIZE"]) * 1024 / F, (agg["FETCH_SIZE"] + agg["WRITE_SIZE"]) * 1024 / F))
for f in glob.glob(O + "/stats/**/*kernel_stats.csv", recursive=True):
    print(open(f).read())
PY
cat $O/summary.txt
grep -h "^tile" $O/*.log | head -3

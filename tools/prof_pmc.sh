#!/bin/bash
# PMC passes over a short bench run (one pass per counter group; gfx950 slot
# limits: 8 SQ, 4 TCC (FETCH_SIZE = 3, WRITE_SIZE = 2), 2 GRBM per pass).
# usage: tools/prof_pmc.sh <outdir> [bench args...]
set -o pipefail
OUT=${1:-gpurun_out/pmc}; shift
ARGS=${@:---sigs 1048576 --steps 2 --warmup 1 --streams 1 --no-cpu --no-latency --no-stream --no-host-fed}
export TMPDIR=/tmp
mkdir -p $OUT
run() { name=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o p -- python3 bench.py $ARGS > $OUT/$name.log 2>&1 || { echo "pass $name failed"; exit 1; }; }
run sq1  SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run sq2  SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS
run fetch FETCH_SIZE
run write WRITE_SIZE
run grbm GRBM_GUI_ACTIVE GRBM_COUNT
echo pmc-done

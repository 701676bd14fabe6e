#!/bin/bash
# k_dsm vs k_dsmp SQ counters (tools/pool_probe.py under rocprofv3 --pmc), two passes.
cd /tmp && export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16 && cd $GRAFT_REPO_ROOT || exit 1
LIB=${LIB:-$PWD/ab/dbg112.so}
FD_AMD_LIB=$LIB timeout -k 10 120 python3 tools/pool_probe.py || exit 1
FD_AMD_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_a -o p -- python3 tools/pool_probe.py > gpurun_out/pmc_a.log 2>&1 || exit 1
FD_AMD_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC --output-format csv -d gpurun_out/pmc_b -o p -- python3 tools/pool_probe.py > gpurun_out/pmc_b.log 2>&1
echo pmc done

#!/bin/bash
# k_dsmp drain-policy A/B: FD_AMD_DIAG builds (per-wave drain clocks, steps and fill after the work
# counter runs out) and plain builds through the bench.  usage: tools/drain_probe.sh dbgA.so dbgB.so -- A.so B.so
export GPU_MAX_HW_QUEUES=16
while [ "$1" != "--" ]; do FD_AMD_LIB=$PWD/$1 timeout -k 10 120 python3 tools/pool_probe.py || exit 1; shift; done
shift
bash tools/ab_libs.sh 2 k_dsmp 2 "$@"

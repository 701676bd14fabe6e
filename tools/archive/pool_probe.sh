#!/bin/bash
# k_dsmp A/B: DBL-step threshold variants (ab/dbg<pct>.so, FD_AMD_DIAG builds)
export GPU_MAX_HW_QUEUES=16
for v in 78 70 88; do FD_AMD_LIB=$PWD/ab/dbg$v.so timeout -k 10 120 python3 tools/pool_probe.py || exit 1; done

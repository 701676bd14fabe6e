#!/bin/bash
# k_dsmp A/B: tail workgroup share (FD_POOL_TAIL_DIV: 1/div of the batch on the per-lane tail path)
export GPU_MAX_HW_QUEUES=16
for div in 0 32 16 8; do FD_POOL_TAIL_DIV=$div FD_AMD_LIB=$PWD/ab/dbg112.so timeout -k 10 120 python3 tools/pool_probe.py || exit 1; done

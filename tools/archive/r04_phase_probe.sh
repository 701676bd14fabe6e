#!/bin/bash
# Round 4: per-phase clocks of k_tile_persist's chunk pipeline (diagnostics library, tools/tile_synth.py;
# where bit 32 = phase clocks) -- gather, prep, decomp, DSM, results per chunk -- and a plain run beside it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 180 python -u tools/tile_synth.py 2048,4,0,0 2048,4,0,32 2048,4,0,40 1024,4,0,32 512,4,0,32 2048,16,1,32 \
  > gpurun_out/r04_phase_probe.jsonl 2> gpurun_out/r04_phase_probe.err
rc=$?
cat gpurun_out/r04_phase_probe.jsonl gpurun_out/r04_phase_probe.err
exit $rc

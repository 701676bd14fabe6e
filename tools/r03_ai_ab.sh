#!/bin/bash
# k_ai4 A/B: gpu parity with the new default, DSM stage of k_ai vs k_ai4 builds (interleaved), and the
# latency kernels' GPU time (their table build moved into a shared helper).
set -o pipefail
O=gpurun_out/r03_ai; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_engine_api_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for lib in ab/ai0.so ab/ai1.so; do
    v=$(FD_AMD_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --no-cpu --no-latency --no-stream --no-host-fed --streams 1 2>>$O/ab.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3f Mv/s  %.3f ms/step  dsm %.3f ms  frac %.4f ok %d' % (d['value']/1e6, d['ms_per_step'], d['stage_ms']['k_dsm'], d['roofline']['frac'], d['verdicts']['ok']))") || { echo "ab failed $lib"; tail -20 $O/ab.err; exit 1; }
    echo "$lib: $v" | tee -a $O/ab.txt
  done
  for lib in ab/t2.so ab/ai1.so; do
    f=$(FD_AMD_LIB=$PWD/$lib timeout -k 10 120 python3 tools/lat_floor.py 2>/dev/null | grep "^4096 " | cut -d' ' -f2-) || exit 1
    echo "$lib lat: $f" | tee -a $O/ab.txt
  done
done

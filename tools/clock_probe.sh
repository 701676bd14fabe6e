#!/bin/bash
# Sample the GPU's power and shader clock while the bench runs (is the
# pipelined bench power-bound?).  usage: tools/clock_probe.sh [bench args...]
O=gpurun_out/clock; mkdir -p $O
timeout -k 10 200 python3 bench.py --no-cpu --no-latency --no-stream "$@" > $O/bench.json 2> $O/bench.err &
B=$!
for i in $(seq 60); do
  kill -0 $B 2>/dev/null || break
  echo "t=$i $(date +%s.%N)" >> $O/smi.txt
  timeout -k 2 5 rocm-smi --showpower --showclocks --showtemp >> $O/smi.txt 2>&1
  sleep 0.5
done
wait $B; echo "bench rc=$?"
cat $O/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value']/1e6, d['ms_per_step'])"
grep -E "Power|sclk|Temperature \(Sensor junction" $O/smi.txt | sort | uniq -c | sort -rn | head -30

#!/bin/bash
# Clock/power while the flagship kernel runs flat out: a long bench in the background, rocm-smi
# samples every ~0.5 s (read-only queries).  Output: gpurun_out/power/*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/power
mkdir -p $o
rocm-smi --showpower --showclocks --showmaxpower > $o/idle.txt 2>&1
timeout -k 10 120 python bench.py --steps 300000 --warmup 400 > $o/bench_long.log 2>&1 &
pid=$!
for i in $(seq 1 40); do
  sleep 0.5
  kill -0 $pid 2>/dev/null || break
  { date +%T.%N; rocm-smi --showpower --showclocks 2>&1 | grep -E "Power|sclk|fclk|mclk"; } >> $o/samples.txt
done
wait $pid
echo "bench rc=$?"
tail -c 600 $o/bench_long.log

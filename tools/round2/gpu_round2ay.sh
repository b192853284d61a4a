#!/bin/bash
# Two-triple (ping-pong) steady loop vs the one-triple loop, step_temporal K = 5..8 and 12, 32768^2, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2ay
mkdir -p $o
: > $o/ab.txt
for rep in 1 2; do
  for K in 5 6 7 8 12; do
    for s2 in 1 0; do
      for bin in base pp; do
        r=$(KB_SPLIT2=$s2 KB_BPC=$((s2 ? 2 : 3)) timeout -k 5 60 ./build/kbench_$bin 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
        echo "$bin K=$K split2=$s2 $r" | sed 's/"skew.*"us_per_gen"/us_per_gen/' | tee -a $o/ab.txt
      done
    done
  done
done

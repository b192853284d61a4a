#!/bin/bash
# Non-temporal row loads (GOL_NT_LOADS) vs plain loads in step_temporal, 32768^2, alternating A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
out=gpurun_out/ntld.txt
: > $out
for rep in 1 2; do
  for K in 1 4 8; do
    for s2 in 0 1; do
      for bin in base ntld; do
        r=$(KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_$bin 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
        echo "$bin K=$K split2=$s2 $r" | tee -a $out
      done
    done
  done
done

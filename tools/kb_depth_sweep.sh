#!/bin/bash
# Per-pass-depth throughput of step_temporal at 32768^2: one tile vs two half-tiles on two streams,
# plan occupancy (waves/SIMD) 2, 3, 4 and the kernel's own maximum.  Each line: us per generation.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for K in 1 2 3 4 5 6 7 8; do
  for bpc in 2 3 4 8; do
    for s2 in 0 1; do
      r=$(KB_BPC=$bpc KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_main 32768 $K $((K*40)) 2>&1 | tail -1)
      echo "K=$K bpc=$bpc split2=$s2 $r"
    done
  done
done

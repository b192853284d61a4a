#!/bin/bash
# K = 9, 10 passes (natural registers: 2 waves/SIMD; capped at 3 waves/SIMD with spills) vs K = 8, 32768^2 two halves.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
out=gpurun_out/k9k10.txt
: > $out
for bin in k10 k10o3; do
  for K in 8 9 10; do
    for bpc in 1 2 3; do
      r=$(KB_BPC=$bpc KB_SPLIT2=1 timeout -k 5 60 ./build/kbench_$bin 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
      echo "$bin K=$K bpc=$bpc split2=1 $r" | tee -a $out
    done
  done
done

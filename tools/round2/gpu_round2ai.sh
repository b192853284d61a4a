#!/bin/bash
# row-major plans: shallow-pass occupancy sweep (waves/SIMD the plan is sized for), one kernel and two halves
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2ai
for K in 1 2 4 5 6 7 8; do for s2 in 0 1; do for bpc in 2 3 4 8; do
  r=$(KB_BPC=$bpc KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_rm 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
  echo "K=$K split2=$s2 bpc=$bpc $r" | tee -a gpurun_out/r2ai/occ.txt | sed 's/"skew.*"rows"/rows/' | cut -c1-130
done; done; done

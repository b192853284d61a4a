#!/bin/bash
# plan order A/B: column-major (default) vs row-major segments, 32768^2, all depths (kbench)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2z
for K in 1 2 4 8; do for s2 in 0 1; do for o in col row; do
  r=$(GOL_PLAN_ORDER=$o KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_po 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
  echo "$o K=$K split2=$s2 $r" | tee -a gpurun_out/r2z/ab.txt | sed 's/"skew.*"us_per_gen"/us_per_gen/' | cut -c1-100
done; done; done
for o in col row; do for a in "8192 24 960 0 0 8 0 4" "16384 8 320"; do
  r=$(GOL_PLAN_ORDER=$o timeout -k 5 60 ./build/kbench_po $a 2>&1 | tail -1) || exit 1
  echo "$o $a $r" | tee -a gpurun_out/r2z/ab.txt | sed 's/"skew.*"us_per_gen"/us_per_gen/' | cut -c1-100
done; done

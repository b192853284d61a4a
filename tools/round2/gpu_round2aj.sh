#!/bin/bash
# temporal-kernel workgroup size (waves per block 1/2/4/8) at 2 and 3 waves/SIMD plans, 32768^2 (kbench, row-major plans)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2aj
run() { # variant bpc K split2
  r=$(KB_BPC=$2 KB_SPLIT2=$4 timeout -k 5 60 ./build/kbench_$1 32768 $3 $(( $3 * 40 )) 2>&1 | tail -1) || exit 1
  echo "$1 bpc=$2 K=$3 split2=$4 $r" | tee -a gpurun_out/r2aj/wpb.txt | sed 's/"skew.*"waves"/waves/' | cut -c1-140
}
for K in 8 4; do for s2 in 0 1; do
  run w4 2 $K $s2; run w4 3 $K $s2
  run w1 8 $K $s2; run w1 12 $K $s2
  run w2 4 $K $s2; run w2 6 $K $s2
  run w8 1 $K $s2
done; done

#!/bin/bash
# n row bands on n streams (n = 1, 2, 3, 4), plan occupancy 2 or 3 waves/SIMD, 32768^2 / 65536^2 K=8 (kbench, row-major plans)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2ad
for N in 32768 65536; do for n in 0 2 3 4; do for bpc in 2 3; do
  r=$(KB_BPC=$bpc KB_SPLIT2=$n timeout -k 5 100 ./build/kbench_sn $N 8 $([ $N = 32768 ] && echo 320 || echo 160) 2>&1 | tail -1) || exit 1
  echo "N=$N parts=$n bpc=$bpc $r" | tee -a gpurun_out/r2ad/splitn.txt | sed 's/"skew.*"us_per_gen"/us_per_gen/' | cut -c1-110
done; done; done

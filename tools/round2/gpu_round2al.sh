#!/bin/bash
# Deep passes (K = 12, 16) vs K = 6..8 at 32768^2, two half-board plans on two streams, plan occupancy 1-3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
out=gpurun_out/deep_k.txt
: > $out
for K in 8 12 16 6; do
  for bpc in 1 2 3; do
    r=$(KB_BPC=$bpc KB_SPLIT2=1 timeout -k 5 60 ./build/kbench_main 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
    echo "K=$K bpc=$bpc split2=1 $r" | tee -a $out
  done
done
for K in 8 12 16; do
  r=$(KB_BPC=3 KB_SPLIT2=0 timeout -k 5 60 ./build/kbench_main 16384 $K $((K*80)) 2>&1 | tail -1) || exit 1
  echo "16384 K=$K bpc=3 $r" | tee -a $out
done

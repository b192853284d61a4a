#!/bin/bash
# shallow-pass diagnosis: stores removed (nost), halo lanes not storing (mst), default (tr); kbench 32768^2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2x
for K in 1 4 8; do for s2 in 0 1; do for v in tr mst nost; do
  r=$(KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_$v 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
  echo "$v K=$K split2=$s2 $r" | tee -a gpurun_out/r2x/ab.txt | sed 's/"skew.*"rows"/rows/' | cut -c1-140
done; done; done

#!/bin/bash
# One kernel per pass over the whole board vs two concurrent half-board kernels (two streams, each a
# one-round plan for the whole GPU, no cross-stream ordering: the timing of two sub-tiles per GPU).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/kb_split2.txt; : > $out
for r in 1 2 3; do
  for sp in 0 1; do
    for b in 3 2; do
      echo "== split2=$sp bpc=$b" >> $out
      KB_SPLIT2=$sp KB_BPC=$b timeout -k 5 60 build/kbench_cur 32768 8 3840 >> $out 2>&1 || exit 3
    done
  done
done
cat $out

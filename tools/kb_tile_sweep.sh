#!/bin/bash
# Tile-kernel sweep at 8192^2 (BASELINE config 2): depth K x waves per workgroup x tile rows, LV=2.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/kb_tile_sweep.txt; : > $out
for K in 16 24 32; do
  for nw in 4 8 16; do
    for rows in 0 34 23; do
      timeout -k 5 60 build/kbench_base 8192 $K 1920 0 0 $nw $rows 2 >> $out 2>&1 || exit 3
    done
  done
done
cat $out

#!/bin/bash
# Temporal kernel: one-round plan vs 2-3 rounds of shorter segments (tail overlap vs more halo).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/kb_rounds.txt; : > $out
for r in 1 2; do
  for rows in 0 45 30 60; do
    echo "== 32768 rows=$rows" >> $out
    timeout -k 5 60 build/kbench_cur 32768 8 1920 0 0 0 $rows >> $out 2>&1 || exit 3
    KB_BPC=2 timeout -k 5 60 build/kbench_cur 32768 8 1920 0 0 0 $rows >> $out 2>&1 || exit 3
  done
done
cat $out

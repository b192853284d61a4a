#!/bin/bash
# Temporal kernel: pass depth K x plan occupancy (waves per SIMD the one-round plan is sized for).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/kb_occ_sweep.txt; : > $out
for N in 16384 32768 65536; do
  g=1920; [ $N = 65536 ] && g=480
  for K in 4 6 8; do
    for b in 1 2 3 4; do
      echo "== N=$N K=$K bpc=$b" >> $out
      KB_BPC=$b timeout -k 5 60 build/kbench_cur $N $K $((g / K * K)) >> $out 2>&1 || exit 3
    done
  done
done
cat $out

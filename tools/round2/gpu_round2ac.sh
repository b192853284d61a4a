#!/bin/bash
# row pitch 514 words (even) vs 528 (128-byte aligned rows), row-major plans (kbench)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2ac
for a in "32768 8 320" "32768 4 160" "32768 1 40" "16384 8 320" "8192 24 960 0 0 8 0 4"; do for s2 in 0 1; do for v in p2 p16; do
  r=$(KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_$v $a 2>&1 | tail -1) || exit 1
  echo "$v split2=$s2 $a $r" | tee -a gpurun_out/r2ac/pitch.txt | sed 's/"skew.*"us_per_gen"/us_per_gen/' | cut -c1-110
done; done; done

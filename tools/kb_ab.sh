#!/bin/bash
# Generic A/B of two kbench builds, alternating on one box: tools/kb_ab.sh <a> <b> [rounds]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/kb_ab_$1_$2.txt; : > $out
for r in $(seq ${3:-3}); do
  for v in $1 $2; do
    echo "== $v" >> $out
    timeout -k 5 60 build/kbench_$v 32768 8 1920 >> $out 2>&1 || exit 3
    timeout -k 5 60 build/kbench_$v 16384 8 1920 >> $out 2>&1 || exit 3
    timeout -k 5 60 build/kbench_$v 65536 8 480 >> $out 2>&1 || exit 3
  done
done
cat $out

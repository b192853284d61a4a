#!/bin/bash
# A/B: DPP lane exchange (kbench_dpp) vs ds_bpermute (kbench_bperm), alternating on one box.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/kb_bperm.txt; : > $out
for v in dpp bperm dpp bperm; do
  echo "== $v" >> $out
  timeout -k 5 60 build/kbench_$v 32768 8 960 >> $out 2>&1 || exit 3
  timeout -k 5 60 build/kbench_$v 32768 8 960 0 1 >> $out 2>&1 || exit 3
  timeout -k 5 60 build/kbench_$v 65536 8 480 >> $out 2>&1 || exit 3
  timeout -k 5 60 build/kbench_$v 8192 24 1920 0 0 8 0 2 >> $out 2>&1 || exit 3
done
cat $out

#!/bin/bash
# Folded tile kernel at 8192^2: levels-per-LDS-pass x waves sweep (kbench), then PMC of the folded
# (K=32, 8 waves, 4 levels) and plain (K=24, the previous auto choice) tile kernels.  One counter set
# per run, --kernel-trace only.  Output: gpurun_out/pmc_fold/*.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/pmc_fold
mkdir -p $o
for k in 24 32; do for nw in 4 8; do for lv in 2 4; do
  echo "fold K=$k nw=$nw lv=$lv $(KB_FOLD=1 timeout -k 5 60 $R/build/kbench_main 8192 $k 960 0 0 $nw 0 $lv | grep -o '"us_per_gen": [0-9.]*')" || exit 1
done; done; done > $o/sweep.txt
cat $o/sweep.txt
pmc() {  # pmc <name> <counters> <env> -- <kbench args>
  local name=$1 ctr=$2 fold=$3; shift 3
  KB_FOLD=$fold timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $ctr -d $o/$name -o $name --output-format csv -- $R/build/kbench_main "$@" > $o/$name.log 2>&1 || { echo "$name failed"; return 1; }
  echo "$name ok"
}
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
B="SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES"
pmc fold_a "$A" 1 8192 32 480 0 0 8 0 4 && pmc fold_b "$B" 1 8192 32 480 0 0 8 0 4 &&
pmc plain_a "$A" 0 8192 24 480 0 0 8 0 4 && pmc plain_b "$B" 0 8192 24 480 0 0 8 0 4 &&
for n in fold_a fold_b plain_a plain_b; do
  f=$(find $o/$n -name '*counter_collection.csv' | head -1)
  echo "== $n"; python3 $R/tools/pmc_summary.py "$f"
done > $o/summary.txt
cat $o/summary.txt

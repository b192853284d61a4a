#!/bin/bash
# Why is a K=7 step_temporal pass nearly as slow as K=8?  PMC of K=6, 7, 8 at 32768^2 (one tile, 3 waves/SIMD plans).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/pmc_k7_after
mkdir -p $o
for K in 7 8 12; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE SQ_WAVE_CYCLES -d $o/k$K -o k$K --output-format csv -- $R/build/kbench_main 32768 $K $((K*24)) > $o/k$K.log 2>&1 || { echo "K=$K failed"; exit 1; }
  f=$(find $o/k$K -name '*counter_collection.csv' | head -1)
  echo "== K=$K $(grep us_per_gen $o/k$K.log | sed 's/.*"rows"/rows/' | cut -c1-120)"
  python3 $R/tools/pmc_summary.py "$f" | grep -A12 step_temporal
done

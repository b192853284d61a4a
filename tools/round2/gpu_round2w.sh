#!/bin/bash
# why a K=1 pass streams at ~55% of the HBM rate: PMC of step_temporal<1> (kbench) vs the column-walk copy (bw_probe)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r2w
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $R/gpurun_out/r2w/a -o a --output-format csv -- $R/build/kbench_tr 32768 1 40 > $R/gpurun_out/r2w/a.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/r2w/b -o b --output-format csv -- $R/build/kbench_tr 32768 1 40 > $R/gpurun_out/r2w/b.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $R/gpurun_out/r2w/c -o c --output-format csv -- $R/build/bw_probe > $R/gpurun_out/r2w/c.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/r2w/d -o d --output-format csv -- $R/build/bw_probe > $R/gpurun_out/r2w/d.log 2>&1 || exit 1
for x in a b c d; do python3 $R/tools/pmc_summary.py $R/gpurun_out/r2w/$x/${x}_counter_collection.csv | grep -A12 "step_temporal<1\|colwalk" | head -30; done

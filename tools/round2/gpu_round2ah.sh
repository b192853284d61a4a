#!/bin/bash
# final rocprof evidence: kernel stats of the driver command and of a 2000-generation run; PMC of the hot kernel
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r2ah
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2ah/d20 -o d20 -- python $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/r2ah/d20.log 2>&1 || { tail -5 $R/gpurun_out/r2ah/d20.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2ah/d2000 -o d2000 -- python $R/bench.py --gpus 1 --steps 2000 --warmup 200 > $R/gpurun_out/r2ah/d2000.log 2>&1 || { tail -5 $R/gpurun_out/r2ah/d2000.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r2ah/pmc -o pmc -- $R/build/kbench_po 32768 8 320 > $R/gpurun_out/r2ah/pmc.log 2>&1 || { tail -5 $R/gpurun_out/r2ah/pmc.log; exit 1; }
ls $R/gpurun_out/r2ah/d20 $R/gpurun_out/r2ah/d2000 $R/gpurun_out/r2ah/pmc

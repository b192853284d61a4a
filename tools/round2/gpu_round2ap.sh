#!/bin/bash
# Kernel trace of the bench with halos through a real 1-rank RCCL communicator (--self-exchange):
# the ncclDevKernel* kernels next to the stencil kernels.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r2ap
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r2ap/prof -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 128 --warmup 16 --self-exchange > $R/gpurun_out/r2ap/bench.log 2>&1 || { tail -20 $R/gpurun_out/r2ap/bench.log; exit 1; }
tail -1 $R/gpurun_out/r2ap/bench.log | cut -c1-400
f=$(find $R/gpurun_out/r2ap/prof -name '*kernel_stats.csv' | head -1)
cp "$f" $R/gpurun_out/r2ap/kernel_stats.csv
cut -c1-160 $R/gpurun_out/r2ap/kernel_stats.csv | head -20

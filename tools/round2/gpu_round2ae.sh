#!/bin/bash
# driver command traced with host markers (GOL_ROCTX=1: gol.run ranges) + kernels: where the timed region's time goes
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r2ae
GOL_ROCTX=1 timeout -k 10 200 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $R/gpurun_out/r2ae/t -o t -- python $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/r2ae/t.log 2>&1 || { tail -5 $R/gpurun_out/r2ae/t.log; exit 1; }
ls $R/gpurun_out/r2ae/t/
tail -1 $R/gpurun_out/r2ae/t.log | cut -c150-260

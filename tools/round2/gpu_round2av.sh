#!/bin/bash
# Kernel trace of a 512-generation bench run (8 supersteps of 64): per-queue gaps at superstep boundaries.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/r2av
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace -d $o/prof -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 512 --warmup 64 > $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
grep '^{"metric"' $o/bench.log | cut -c1-200
f=$(find $o/prof -name '*kernel_trace.csv' | head -1)
cp $f $o/kernel_trace.csv
python3 $R/tools/trace_queues.py $o/kernel_trace.csv --last-us 5400 > $o/queues.txt
cat $o/queues.txt | tail -60

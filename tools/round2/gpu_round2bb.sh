#!/bin/bash
# Kernel traces of 8 driver-command runs (12 + 8 cut): the timed region's kernels per queue, to see what the slow runs do.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/r2bb
mkdir -p $o
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d $o/p$i -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $o/b$i.log 2>&1 || { tail -5 $o/b$i.log; exit 1; }
  f=$(find $o/p$i -name '*kernel_trace.csv' | head -1)
  v=$(grep '^{"metric"' $o/b$i.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print("%.3f" % (d["ms_per_step"]*1e3))')
  echo "== run $i: $v us/gen"
  python3 $R/tools/trace_queues.py $f --last-us 600 --show 8 | grep -v "^  busy" | head -24
done > $o/summary.txt
grep "== run" $o/summary.txt

#!/bin/bash
# GPU batch G (round 4): kernel traces of the driver's timed run, the default schedule and the flow
# schedule (one dispatch per superstep), summarised by tools/timed_trace.py.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp GOL_ROCTX=1
for s in auto flow; do
  rm -rf gpurun_out/trace_$s; mkdir -p gpurun_out/trace_$s
  for i in 1 2; do
    GOL_SCHEDULE=$s timeout -k 10 180 rocprofv3 --kernel-trace --marker-trace --output-format csv -d gpurun_out/trace_$s/r$i -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-phases > gpurun_out/trace_$s/b$i.log 2>&1 || { echo "trace $s rc=$?"; tail -5 gpurun_out/trace_$s/b$i.log; exit 1; }
    echo "== schedule $s run $i" >> gpurun_out/trace_summary.txt
    python3 tools/timed_trace.py gpurun_out/trace_$s/r$i >> gpurun_out/trace_summary.txt 2>&1
  done
done
cat gpurun_out/trace_summary.txt

#!/bin/bash
# GPU: kernel traces of the driver's cut through the RCCL self-exchange (a rank with neighbours on one
# GPU), summarised by tools/timed_trace.py (RCCL's kernels included).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/trace_selfx
export TMPDIR=/tmp GOL_ROCTX=1
: > gpurun_out/trace_selfx/summary.txt
for i in 1 2; do
  timeout -k 10 180 rocprofv3 --kernel-trace --marker-trace --output-format csv -d gpurun_out/trace_selfx/r$i -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange --no-phases > gpurun_out/trace_selfx/b$i.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/trace_selfx/b$i.log; exit 1; }
  echo "== run $i" >> gpurun_out/trace_selfx/summary.txt
  python3 tools/timed_trace.py gpurun_out/trace_selfx/r$i >> gpurun_out/trace_selfx/summary.txt 2>&1
done
cat gpurun_out/trace_selfx/summary.txt

#!/bin/bash
# GPU batch (round 4): flow kernel checks, GPU tests, the 32768^2 cut sweep, the driver's bench A/B
# (auto vs forced flow) and a kernel trace of the flow bench.  Every step has its own time limit; the
# batch stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "[batch] $(date +%T) $*"; }
step flowbench-small
timeout -k 10 60 build/flowbench 4096 2,2 5 1.0 > gpurun_out/fb_small.txt 2>&1 || { echo "flowbench small rc=$?"; cat gpurun_out/fb_small.txt; exit 1; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_rccl.py tests/test_gpu_resident.py -x -v \
    --timeout 180 --timeout-method thread -k "flow or registered or timeout" > gpurun_out/test_flow.txt 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/test_flow.txt; exit 1; }
step sweep
bash tools/flow_sweep.sh gpurun_out/flow_sweep.txt || exit 1
step bench-ab
bash tools/flow_bench_ab.sh gpurun_out/flow_bench_ab.jsonl 5 > gpurun_out/flow_bench_ab.txt 2>&1 || { cat gpurun_out/flow_bench_ab.txt; exit 1; }
step trace
GOL_SCHEDULE=flow GOL_ROCTX=1 timeout -k 10 240 rocprofv3 --kernel-trace --marker-trace --stats -d gpurun_out/prof_flow -o flow -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-phases > gpurun_out/prof_flow_bench.txt 2>&1 || { echo "trace rc=$?"; tail -20 gpurun_out/prof_flow_bench.txt; exit 1; }
python3 tools/timed_trace.py gpurun_out/prof_flow > gpurun_out/prof_flow_timed.txt 2>&1 || true
step done

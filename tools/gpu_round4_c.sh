#!/bin/bash
# GPU batch C (round 4): launch-latency probe, the flow GPU tests (tile fallback, flow+ov on the
# CU-restricted stream, forced flow on small boards), then batch B (configs with flow A/B,
# self-exchange, rehearsal, PMC).  Each step has its own time limit; the batch stops at a failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "[batch-c] $(date +%T) launch probe"
timeout -k 10 120 build/launch_probe 64 > gpurun_out/launch_probe.txt 2>&1 || { echo "launch_probe rc=$?"; exit 1; }
echo "[batch-c] $(date +%T) flow tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_rccl.py -x -v --timeout 180 --timeout-method thread \
    -k "flow or registered" > gpurun_out/test_flow.txt 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/test_flow.txt; exit 1; }
tail -3 gpurun_out/test_flow.txt
bash tools/gpu_round4_b.sh

#!/bin/bash
# GPU: step_flow checks — flowbench on a small board, the flow GPU tests, then the 32768^2 cut sweep.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 build/flowbench 4096 2,2 5 1.0 > gpurun_out/fb_small.txt 2>&1 || { echo "flowbench small rc=$?" >> gpurun_out/fb_small.txt; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_rccl.py tests/test_gpu_resident.py -x -v \
    --timeout 180 --timeout-method thread -k "flow or registered or timeout" > gpurun_out/test_flow.txt 2>&1 || { echo "pytest rc=$?" >> gpurun_out/test_flow.txt; exit 1; }
bash tools/flow_sweep.sh gpurun_out/flow_sweep2.txt

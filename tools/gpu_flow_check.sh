set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 build/flowbench 4096 2,2 5 1.0 > gpurun_out/fb_small.txt 2>&1 || { echo "flowbench small rc=$?" >> gpurun_out/fb_small.txt; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_flow.py -x -v --timeout 120 --timeout-method thread > gpurun_out/test_flow.txt 2>&1 || { echo "pytest rc=$?" >> gpurun_out/test_flow.txt; exit 1; }
bash tools/flow_sweep.sh gpurun_out/flow_sweep2.txt

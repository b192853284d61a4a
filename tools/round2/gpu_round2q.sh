#!/bin/bash
# in-place LDS tile (one buffer, private halo copies) vs double-buffered: correctness (tile tests) + kbench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2q
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_cli.py -x -q -m gpu -k "tile or auto or cfg or perf" --timeout 120 --timeout-method thread > gpurun_out/r2q/pytest.log 2>&1 || { tail -30 gpurun_out/r2q/pytest.log; exit 1; }
tail -1 gpurun_out/r2q/pytest.log
for shape in "8192 8192" "16384 16384" "4096 32768" "32768 32768"; do set -- $shape; N=$1; W=$2
  for K in 16 24 32; do for lv in 2 4; do for ip in 0 1; do
    r=$(KB_W=$W KB_INPLACE=$ip timeout -k 5 60 ./build/kbench_tl $N $K $((K*40)) 0 0 8 0 $lv 2>&1 | tail -1) || exit 1
    echo "N=$N W=$W K=$K lv=$lv inplace=$ip $r" | tee -a gpurun_out/r2q/inplace_ab.txt | sed 's/"skew.*"rows"/rows/' | cut -c1-150
  done; done; done
done
for i in 1 2; do timeout -k 10 60 ./build/gol 5 8192 1000 256 0 | head -1; done
timeout -k 10 150 python bench.py --gpus 1 --steps 1000 --warmup 100 --size 4096 --width 32768 > gpurun_out/r2q/s3_local.log 2>&1 || exit 1; tail -1 gpurun_out/r2q/s3_local.log | cut -c170-600
timeout -k 10 150 python bench.py --gpus 1 --steps 1000 --warmup 100 --size 16384 > gpurun_out/r2q/b16k.log 2>&1 || exit 1; tail -1 gpurun_out/r2q/b16k.log | cut -c170-600

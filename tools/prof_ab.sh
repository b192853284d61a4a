#!/bin/bash
# Kernel-trace A/B: the standalone kbench timing loop vs the engine (bench.py) on the same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kb -o kb --output-format csv -- build/kbench_tile 32768 8 960 > gpurun_out/prof_kb.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench --output-format csv -- python3 bench.py --steps 2000 --warmup 200 > gpurun_out/prof_bench.log 2>&1 || exit 3
grep -h step_temporal gpurun_out/prof_kb/kb_kernel_stats.csv gpurun_out/prof_bench/bench_kernel_stats.csv

#!/bin/bash
# Driver-style bench (bench.py --gpus 1 --steps 20 --warmup 5) three times, then a kernel trace of
# the same command (per-dispatch timeline of the timed region).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dtrace
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/dtrace/bench_$i.json 2> gpurun_out/dtrace/bench_$i.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/dtrace/bench_$i.json')); print('run $i', d['ms_per_step']*1e3, 'us/gen', d['config']['schedule'])"
done
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dtrace/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/dtrace/prof.log 2>&1

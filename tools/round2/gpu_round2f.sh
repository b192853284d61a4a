#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2f
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2f/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/r2f/$name.log" | cut -c1-700
  return $rc
}
run headline 300 python -u -m pytest tests/test_gpu_headline.py -x -v -m gpu --timeout 280 --timeout-method thread || exit $?
run pytest_engine 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py -x -q -m gpu --timeout 120 --timeout-method thread || exit $?
for i in 1 2 3; do run bench_$i 120 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?; done
run bench_long 200 python bench.py --gpus 1 --steps 2000 --warmup 200 || exit $?
run bench_self 200 python bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange || exit $?
run bench_self_long 200 python bench.py --gpus 1 --steps 2000 --warmup 200 --self-exchange || exit $?

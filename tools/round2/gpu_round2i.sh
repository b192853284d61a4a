#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2i
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2i/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 1 "gpurun_out/r2i/$name.log" | cut -c150-260
  return $rc
}
for i in 1 2 3 4 5; do run bench_$i 120 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?; done
run pytest_sub 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py -k "subtiles or hint" -x -q -m gpu --timeout 120 --timeout-method thread || exit $?

#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2d
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2d/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/r2d/$name.log" | cut -c1-2500
  return $rc
}
run pytest_engine 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py -x -q -m gpu --timeout 120 --timeout-method thread || exit $?
for i in 1 2 3; do run bench_$i 120 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?; done
run short 300 python tools/short_run_probe.py --variants sub2,sub0 || exit $?
run bench_long 200 python bench.py --gpus 1 --steps 2000 --warmup 200 || exit $?
run prof 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2d/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5

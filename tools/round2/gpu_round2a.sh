#!/bin/bash
# Round-2 GPU session A: RCCL self-probe (teardown variants), RCCL self-exchange tests, engine
# suite, driver-style bench + kernel trace.  Every GPU step has its own limit; a crash/timeout ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2a
export TMPDIR=/tmp
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2a/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 6 "gpurun_out/r2a/$name.log"
  return $rc
}
#run probe_eager_only 40 ./build/rccl_self_probe 1
#run probe_graph 40 ./build/rccl_self_probe 0
run pytest_rccl 300 python -u -m pytest tests/test_gpu_rccl.py -x -v -m gpu --timeout 120 --timeout-method thread || exit $?
run pytest_engine 600 python -u -m pytest tests/test_gpu_engine.py -x -q -m gpu --timeout 120 --timeout-method thread || exit $?
for i in 1 2 3; do
  run bench_$i 120 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
done
run bench_long 200 python bench.py --gpus 1 --steps 2000 --warmup 200 || exit $?
run bench_self_rccl 200 python bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange || exit $?
run prof 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2a/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5

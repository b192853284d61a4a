#!/bin/bash
# round 2 re-entry: full GPU suite + driver bench + kernel trace of the driver bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2j
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2j/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "gpurun_out/r2j/$name.log" | cut -c1-400
  return $rc
}
run pytest_all 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread || exit $?
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
for i in 1 2; do run bench_$i 120 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?; done
run prof 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2j/prof -o bench -- python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?

#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2g
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2g/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 1 "gpurun_out/r2g/$name.log" | cut -c1-400
  return $rc
}
for i in 1 2 3 4; do run bench_$i 120 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?; done
run prof 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2g/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5

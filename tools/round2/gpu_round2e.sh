#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2e
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2e/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "gpurun_out/r2e/$name.log" | cut -c1-600
  return $rc
}
run prof_graph 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2e/prof_graph -o run -- python3 bench.py --gpus 1 --steps 256 --warmup 5 || exit $?
GOL_GRAPH=0 run prof_eager 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2e/prof_eager -o run -- python3 bench.py --gpus 1 --steps 256 --warmup 5 || exit $?
run short 300 python tools/short_run_probe.py --variants sub2,sub0,sub2-nograph,sub0-nograph || exit $?
run short256 300 python tools/short_run_probe.py --steps 256 --reps 5 --variants sub2,sub0,sub2-nograph,sub0-nograph || exit $?

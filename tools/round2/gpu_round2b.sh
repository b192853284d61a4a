#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2b
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2b/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 8 "gpurun_out/r2b/$name.log"
  return $rc
}
run short 300 python tools/short_run_probe.py --variants sub2,sub0,sub2-nograph,sub0-nograph,sub0-r32 || exit $?
run short_torch 200 python tools/short_run_probe.py --variants sub2,sub0 --torch-sync || exit $?
GOL_SUBTILES=2 run prof_self_sub 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2b/prof_self_sub -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 5 --self-exchange

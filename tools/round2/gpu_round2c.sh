#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2c
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/r2c/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/r2c/$name.log" | cut -c1-1500
  return $rc
}
run self_rccl 200 python bench.py --gpus 1 --steps 640 --warmup 64 --self-exchange || exit $?
GOL_SUBTILES=2 run prof_self_sub 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2c/prof_self_sub -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 5 --self-exchange || exit $?
run short 300 python tools/short_run_probe.py --variants sub2,sub0 || exit $?
run kbsweep 400 bash tools/kb_depth_sweep.sh

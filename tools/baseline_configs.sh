#!/bin/bash
# BASELINE.json configs that fit one MI355X (configs 3/4 at 8 GPUs are run by the driver's scaling
# bench; here their boards run on one GPU).  Each GPU step has its own time limit; a fatal status
# (timeout, abort, segfault) ends the script.  Output: gpurun_out/configs/*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/configs
mkdir -p $out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 4 "$out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "FATAL rc=$rc in $name, stopping"; exit $rc; fi
  return 0
}
for c in "$@"; do
  case $c in
    cfg1) step cfg1_cpu_256 120 env GOL_BACKEND=cpu ./build/gol 5 256 100 256 0 ;;
    cfg2) step cfg2_cli_8192 120 env GOL_BACKEND=hip ./build/gol 5 8192 1000 256 0 ;;
    cfg2b) step cfg2_bench_8192 120 python bench.py --size 8192 --steps 1000 --warmup 100 ;;
    cfg3) step cfg3_bench_32768 300 python bench.py --size 32768 --steps 2000 --warmup 200 ;;
    cfg4) step cfg4_bench_65536_2d 300 python bench.py --size 65536 --scaling strong --decomp 2d --steps 400 --warmup 40 ;;
    cfg5) step cfg5_capacity_1048576 600 python bench.py --size 1048576 --steps 16 --warmup 8 ;;
    cfg5b) step cfg5_capacity_786432 600 python bench.py --size 786432 --steps 16 --warmup 8 ;;
    *) echo "unknown config $c"; exit 2 ;;
  esac
done

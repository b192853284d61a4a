#!/bin/bash
# One GPU-box session: GPU tests, smoke, short bench, kernel profile.  Every GPU step has its own
# time limit; a crash/abort/timeout (rc >= 124) ends the script, plain test failures (rc 1) do not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "FATAL rc=$rc in $name, stopping"; exit $rc; fi
  return 0
}
rocminfo 2>/dev/null | grep -m3 -E "Marketing|gfx950|Compute Unit" > gpurun_out/rocminfo.txt
for s in "$@"; do
  case $s in
    tests)  step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  step bench 600 python bench.py --steps 2000 --warmup 200 --yardstick ;;
    prof)   step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof --output-format csv -- python3 bench.py --steps 400 --warmup 40 ;;
    *)      step custom 600 bash -c "$s" ;;
  esac
done

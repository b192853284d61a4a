#!/bin/bash
# Round-6 GPU batches on one MI355X.  Every GPU step has its own time limit; a fatal status (fault,
# abort, segfault, time limit) ends the script.  Output: gpurun_out/r6/<batch>/ (summary.txt).
#   tools/round6.sh <batch>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B=$1
O=gpurun_out/r6/$B; mkdir -p $O
S=$O/summary.txt; : > $S
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
pyt() {  # pyt <log> <pytest args...>
  local log=$1; shift
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread "$@" > $O/$log 2>&1; local rc=$?
  echo "== pytest $* rc=$rc: $(tail -1 $O/$log)" >> $S; return $rc
}
reps() {  # reps <n> <variants...>: tools/bench_reps.sh, lines appended to the summary
  rm -f gpurun_out/bench_reps.txt
  tools/bench_reps.sh "$@" > /dev/null; local rc=$?
  cat gpurun_out/bench_reps.txt >> $S; cat gpurun_out/bench_reps.jsonl >> $O/bench.jsonl 2>/dev/null
  rm -f gpurun_out/bench_reps.txt gpurun_out/bench_reps.jsonl; return $rc
}
case $B in
b1)
  # the round-6 tests first (ADVICE fixes, the capture guard, the prediction without a snapshot)
  pyt new_tests.log tests/test_gpu_rccl.py tests/test_gpu_engine.py -k "unaligned_width or capture_refused or without_snapshot or split_pipe" || exit 1
  reps 3 "" "--self-exchange" || exit 1
  # the forked-stream RCCL capture: the origin-stream and eager forms first, the crashing form last
  for m in eager origin+reg fork fork+reg; do
    timeout -k 10 120 build/rccl_capture_probe $m > $O/capture_$m.log 2>&1; rc=$?
    echo "== rccl_capture_probe $m rc=$rc: $(tail -1 $O/capture_$m.log)" >> $S
    fatal $rc && break
  done
  ;;
*) echo "unknown batch $B"; exit 2 ;;
esac
cat $S

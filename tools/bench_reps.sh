#!/bin/bash
# GPU: repeated bench runs of several variants, interleaved, one summary line per run.
#   tools/bench_reps.sh <reps> "<env and args A>" ["<env and args B>" ...]
# Leading VAR=value words of a variant go to the environment, the rest to bench.py (after the driver's
# defaults --gpus 1 --steps 20 --warmup 5, which later arguments override).  Summary lines go to stdout
# and gpurun_out/bench_reps.txt; the full JSON of every run to gpurun_out/bench_reps.jsonl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
reps=$1; shift
o=gpurun_out/bench_reps.txt
j=gpurun_out/bench_reps.jsonl
run() {  # run <variant>
  local envs=() args=()
  for w in $1; do if [[ $w == *=* && ${#args[@]} -eq 0 ]]; then envs+=("$w"); else args+=("$w"); fi; done
  env "${envs[@]}" timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 "${args[@]}" 2>>gpurun_out/bench_reps.err
}
for i in $(seq 1 "$reps"); do
  for v in "$@"; do
    r=$(run "$v") || { echo "bench rc=$? ($v)"; exit 1; }
    echo "$r" >> $j
    echo "$r" | python3 tools/bench_line.py "$v" | tee -a $o
  done
done

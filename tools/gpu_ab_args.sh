#!/bin/bash
# GPU: the driver's bench command alternating two argument / environment variants, N pairs on one box.
#   tools/gpu_ab_args.sh <pairs> "<env and args A>" "<env and args B>"   (e.g. "X=1 --watchdog 0")
set -o pipefail
cd "$(dirname "$0")/.."
pairs=$1; A=$2; B=$3
o=gpurun_out/ab_args.txt
: > $o
run() {  # run <variant>: leading VAR=value words go to env, the rest to bench.py
  local envs=() args=()
  for w in $1; do if [[ $w == *=* && ${#args[@]} -eq 0 ]]; then envs+=("$w"); else args+=("$w"); fi; done
  env "${envs[@]}" timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 "${args[@]}" 2>/dev/null
}
for i in $(seq 1 $pairs); do
  for v in "$A" "$B"; do
    r=$(run "$v") || { echo "bench rc=$? ($v)"; exit 1; }
    echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$v] %.3f us/gen' % (d['ms_per_step']*1e3), d['config']['schedule'])" | tee -a $o
  done
done

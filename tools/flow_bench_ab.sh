#!/bin/bash
# GPU: the driver's bench command, alternating the default schedule choice (auto) with forced flow
# supersteps, N pairs; one JSON line per run in $out, a summary line per run on stdout.
# Usage: tools/flow_bench_ab.sh [out=gpurun_out/flow_bench_ab.jsonl] [pairs=5] [extra bench args...]
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/flow_bench_ab.jsonl}
pairs=${2:-5}
shift 2
mkdir -p "$(dirname "$out")"
for i in $(seq 1 "$pairs"); do
  for mode in auto flow; do
    if [ "$mode" = auto ]; then env_sched=""; else env_sched="GOL_SCHEDULE=flow"; fi
    line=$(env $env_sched timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 "$@" 2>gpurun_out/bench_ab_err.txt | grep '^{') || { echo "bench failed ($mode)"; cat gpurun_out/bench_ab_err.txt; exit 1; }
    echo "{\"mode\": \"$mode\", \"run\": $line}" >> "$out"
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('$mode', round(d['ms_per_step']*1e3,3), 'us/gen', d['config']['schedule'], d['config']['kernel'])" "$line"
  done
done

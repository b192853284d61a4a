#!/bin/bash
# Config 2 board: bench.py at 1000 vs 2000 timed steps and the CLI, alternating (fixed per-run cost of the bench path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cfg2steps
for rep in 1 2; do
  for st in 1000 2000; do
    timeout -k 10 120 python bench.py --size 8192 --steps $st --warmup 100 > gpurun_out/cfg2steps/b.log 2>&1 || exit 3
    grep '^{' gpurun_out/cfg2steps/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('bench steps=$st', round(d['ms_per_step']*1e3,4), 'us/gen', 'graph_launches', c['graph_launches'])"
  done
  timeout -k 10 120 ./build/gol 5 8192 1000 256 0 | grep TOTAL || exit 3
done | tee gpurun_out/cfg2steps/ab.txt

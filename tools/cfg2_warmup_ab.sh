#!/bin/bash
# bench.py at 8192^2, 1000 timed steps, warmup 0 / 96 / 100 / 200 (graph parity and eager remainders before the timed run).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cfg2steps
for rep in 1 2; do
  for w in 0 96 100 200; do
    timeout -k 10 120 python bench.py --size 8192 --steps 1000 --warmup $w > gpurun_out/cfg2steps/w.log 2>&1 || exit 3
    grep '^{' gpurun_out/cfg2steps/w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('warmup=$w', round(d['ms_per_step']*1e3,4), 'us/gen', 'graph_launches', c['graph_launches'])"
  done
done | tee gpurun_out/cfg2steps/warmup_ab.txt

#!/bin/bash
# Split-schedule cost vs halo depth R (GOL_FORCE_SPLIT=1, eager supersteps as on multi-GPU runs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/split_cost
mkdir -p $o
for R in 32 48 64; do
  timeout -k 10 180 env GOL_FORCE_SPLIT=1 python bench.py --steps 4000 --warmup 400 --halo-depth $R --no-graph > $o/split_r$R.log 2>&1 || exit 3
  python3 -c "import json; d=json.loads([l for l in open('$o/split_r$R.log') if l.startswith('{')][-1]); c=d['config']; print('R=$R %.4e %.3f us/gen kernel=%s' % (d['value'], d['ms_per_step']*1e3, c['kernel']))"
done

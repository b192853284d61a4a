#!/bin/bash
# Pass order of a short superstep (GOL_PASS_ORDER=asc: 4 + 8 + 8 instead of 8 + 8 + 4), driver command, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2au
mkdir -p $o
for rep in 1 2 3; do
  for ord in desc asc; do
    timeout -k 10 120 env GOL_PASS_ORDER=$ord python bench.py --gpus 1 --steps 20 --warmup 5 > $o/${ord}_$rep.log 2>&1 || exit 1
    grep '^{"metric"' $o/${ord}_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); print("'$ord': %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]))'
  done
done

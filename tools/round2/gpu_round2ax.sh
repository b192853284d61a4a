#!/bin/bash
# Unequal sub-tile halves (GOL_SUB_SPLIT per mille for half 0, which runs ahead): 20 and 2000 steps, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2ax
mkdir -p $o
for rep in 1 2; do
  for steps in 20 2000; do
    for f in 500 520 540; do
      timeout -k 10 120 env GOL_SUB_SPLIT=$f python bench.py --gpus 1 --steps $steps --warmup 5 > $o/f${f}_${steps}_$rep.log 2>&1 || exit 1
      grep '^{"metric"' $o/f${f}_${steps}_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); print("split '$f' steps '$steps': %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]))'
    done
  done
done

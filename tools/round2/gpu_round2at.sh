#!/bin/bash
# Does the GPU clock ramp matter for the driver's 20-step timed region?  --warmup 5 (driver) vs a
# 2000-generation warmup that keeps the GPU busy until just before the timed steps.  Alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2at
mkdir -p $o
for rep in 1 2 3; do
  for w in 5 2000; do
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup $w > $o/w${w}_$rep.log 2>&1 || exit 1
    grep '^{"metric"' $o/w${w}_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); print("warmup '$w': %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]))'
  done
done

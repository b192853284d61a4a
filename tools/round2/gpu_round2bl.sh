#!/bin/bash
# Sub-tile superstep length: halo depth 64 (auto) vs 128 vs 96, 2000 steps, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2bl
mkdir -p $o
for rep in 1 2; do
  for R in 64 128 96; do
    timeout -k 10 150 python bench.py --gpus 1 --steps 2048 --warmup 128 --halo-depth $R > $o/r${R}_$rep.log 2>&1 || exit 1
    grep '^{"metric"' $o/r${R}_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("R='$R' %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]), c["schedule"], c["halo_depth"])'
  done
done

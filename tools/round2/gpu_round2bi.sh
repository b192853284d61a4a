#!/bin/bash
# 20-step runs with halos through RCCL self-exchange: sub-tile exchange overlap off / on, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2bi
mkdir -p $o
for i in 1 2 3; do
  for ov in 0 1; do
    timeout -k 10 150 env GOL_SUBTILE_OVERLAP=$ov python bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange > $o/ov${ov}_$i.log 2>&1 || exit 1
    grep '^{"metric"' $o/ov${ov}_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("ov'$ov' %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]), c["schedule"])'
  done
done

#!/bin/bash
# One-tile strips with neighbours (RCCL self-exchange): halo depth 64 (auto) vs 128, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2bn
mkdir -p $o
for rep in 1 2; do
  for R in 64 128; do
    for cfg in "s3 --size 4096 --width 32768" "c4_1d --size 8192 --width 65536" "s2 --size 16384 --width 32768"; do
      set -- $cfg; n=$1; shift
      timeout -k 10 150 python bench.py --gpus 1 --steps 1280 --warmup 128 --self-exchange --halo-depth $R "$@" > $o/${n}_$R_$rep.log 2>&1 || exit 1
      grep '^{"metric"' $o/${n}_$R_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("'$n' R='$R' %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]), c["schedule"], c["halo_depth"])'
    done
  done
done

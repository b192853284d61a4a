#!/bin/bash
# Sub-tile events with a device-scope release (GOL_SUB_EVENT_SCOPE=device) vs system scope, alternating:
# 20 steps with RCCL self-exchange (one exchange + cross-queue wait per run), 20 steps local, 2048 steps local.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2bs
mkdir -p $o
for rep in 1 2 3; do
  for sc in system device; do
    for cfg in "self20 --steps 20 --warmup 5 --self-exchange" "loc20 --steps 20 --warmup 5" "loc2k --steps 2048 --warmup 128"; do
      set -- $cfg; n=$1; shift
      timeout -k 10 150 env GOL_SUB_EVENT_SCOPE=$sc python bench.py --gpus 1 "$@" > $o/${n}_${sc}_$rep.log 2>&1 || exit 1
      grep '^{"metric"' $o/${n}_${sc}_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); print("'$n' '$sc' %.3f us/gen" % (d["ms_per_step"]*1e3))'
    done
  done
done

#!/bin/bash
# RCCL launch knobs vs the exchange cost of a 20-step run through RCCL self-exchange, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2bt
mkdir -p $o
for rep in 1 2 3; do
  for v in default mix0 lo1; do
    case $v in default) e="GOL_X=1";; mix0) e="NCCL_GRAPH_MIXING_SUPPORT=0";; lo1) e="NCCL_LAUNCH_ORDER_IMPLICIT=1";; esac
    timeout -k 10 150 env $e python bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange > $o/${v}_$rep.log 2>&1 || { tail -3 $o/${v}_$rep.log; exit 1; }
    grep '^{"metric"' $o/${v}_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); print("'$v' %.3f us/gen" % (d["ms_per_step"]*1e3))'
  done
done

#!/bin/bash
# Cost of the multi-GPU superstep structure on one GPU (GOL_FORCE_SPLIT=1: interior/boundary split,
# comm stream and cross-stream events with an empty exchange), eager vs graph-replayed, 32768^2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/split_cost
mkdir -p $o
run() {  # run <name> <env...> -- <bench args>
  local name=$1; shift
  timeout -k 10 180 env "$@" > $o/$name.log 2>&1
  local rc=$?
  python3 -c "import json,sys; d=json.loads([l for l in open('$o/$name.log') if l.startswith('{')][-1]); c=d['config']; print('%-22s %.4e  %.3f us/gen  sched=%s kernel=%s graphs=%s' % ('$name', d['value'], d['ms_per_step']*1e3, c['schedule'], c['kernel'], c['graph_launches']))" || { echo "$name rc=$rc"; tail -5 $o/$name.log; }
  [ $rc -ge 124 ] && exit $rc
  return 0
}
B="python bench.py --steps 4000 --warmup 400 --halo-depth 32"
run unsplit_graph   GOL_FORCE_SPLIT=0 $B
run unsplit_eager   GOL_FORCE_SPLIT=0 $B --no-graph
run split_graph     GOL_FORCE_SPLIT=1 $B
run split_eager     GOL_FORCE_SPLIT=1 $B --no-graph
run split_eager_devscope GOL_FORCE_SPLIT=1 GOL_EVENT_SCOPE=device $B --no-graph

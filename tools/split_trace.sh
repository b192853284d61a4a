#!/bin/bash
# Kernel timelines of the interior/boundary edge schedule on one GPU (GOL_FORCE_SPLIT=1).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/split
mkdir -p $o
run() {  # run <name> <env...>
  local name=$1; shift
  timeout -k 10 300 env "$@" rocprofv3 --kernel-trace -d $o/$name -o $name --output-format csv -- python3 $R/bench.py --steps 400 --warmup 40 > $o/$name.log 2>&1 || exit $?
}
run nosplit GOL_FORCE_SPLIT=0
run split_graph GOL_FORCE_SPLIT=1
run split_nograph GOL_FORCE_SPLIT=1 GOL_GRAPH=0
run split_nograph_nomask GOL_FORCE_SPLIT=1 GOL_GRAPH=0 GOL_EDGE_CUS=0

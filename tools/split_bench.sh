#!/bin/bash
# Host-timed bench of the split (multi-GPU) schedule on one GPU, no profiler.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/split_bench; mkdir -p $o
for v in "nosplit:GOL_FORCE_SPLIT=0" "split_auto:GOL_FORCE_SPLIT=1" "split_temporal:GOL_FORCE_SPLIT=1 GOL_KERNEL=temporal" \
         "split_nograph:GOL_FORCE_SPLIT=1 GOL_GRAPH=0" "edge8:GOL_FORCE_SPLIT=1 GOL_EDGE_CUS=8" \
         "split_auto_8192:GOL_FORCE_SPLIT=1 --size 8192" "nosplit_8192:GOL_FORCE_SPLIT=0 --size 8192"; do
  name=${v%%:*}; rest=${v#*:}
  envs=$(echo $rest | tr ' ' '\n' | grep '=' | tr '\n' ' '); args=$(echo $rest | tr ' ' '\n' | grep -v '=' | tr '\n' ' ')
  timeout -k 10 300 env $envs python bench.py --steps 2000 --warmup 200 $args > $o/$name.log 2>&1 || exit $?
  echo "$name $(grep -o '"value": [0-9.e+]*\|"kernel": "[^"]*"' $o/$name.log | tr '\n' ' ')"
done

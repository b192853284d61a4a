#!/bin/bash
# Host-timed bench of the split (multi-GPU) schedule on one GPU, no profiler.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/split_bench; mkdir -p $o
for v in "nosplit:GOL_FORCE_SPLIT=0" "split_R8:GOL_FORCE_SPLIT=1 GOL_HALO_DEPTH=8" \
         "split_R32K8:GOL_FORCE_SPLIT=1 GOL_HALO_DEPTH=32 GOL_KERNEL_DEPTH=8" \
         "split_R64K8:GOL_FORCE_SPLIT=1 GOL_HALO_DEPTH=64 GOL_KERNEL_DEPTH=8" \
         "nosplit_R32K8:GOL_FORCE_SPLIT=0 GOL_HALO_DEPTH=32 GOL_KERNEL_DEPTH=8" \
         "split_R32K8_8192:GOL_FORCE_SPLIT=1 GOL_HALO_DEPTH=32 GOL_KERNEL_DEPTH=8 --size 8192" \
         "nosplit_8192:GOL_FORCE_SPLIT=0 --size 8192"; do
  name=${v%%:*}; rest=${v#*:}
  envs=$(echo $rest | tr ' ' '\n' | grep '=' | tr '\n' ' '); args=$(echo $rest | tr ' ' '\n' | grep -v '=' | tr '\n' ' ')
  timeout -k 10 300 env $envs python bench.py --steps 2048 --warmup 256 $args > $o/$name.log 2>&1 || exit $?
  echo "$name $(grep -o '"value": [0-9.e+]*\|"kernel": "[^"]*"' $o/$name.log | tr '\n' ' ')"
done

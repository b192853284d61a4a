#!/bin/bash
# Build kbench variants: build/kbench_<name> for each "name:flags" argument.
cd "$(dirname "$0")/.."
SRC="tools/kbench.cpp csrc/src/hip/step_kernels.hip csrc/src/hip/pipe_kernel.hip csrc/src/hip/aux_kernels.hip csrc/src/core/plan.cpp csrc/src/core/geometry.cpp csrc/src/core/config.cpp"
pids=()
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  [ "$name" = "$spec" ] && flags=""
  ( hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/include -Wno-unused-result -Wno-unused-value $flags $SRC \
      -o build/kbench_$name 2>&1 | grep -E "error" ; echo "built kbench_$name" ) &
  pids+=($!)
done
wait

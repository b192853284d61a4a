#!/bin/bash
# Build build/flowbench (tools/flowbench.cpp): the step_flow kernel against step_temporal passes.
cd "$(dirname "$0")/.."
mkdir -p build/fb
SRCS="csrc/src/hip/flow_kernel.hip csrc/src/hip/step_kernels.hip csrc/src/hip/aux_kernels.hip"
objs=()
for s in $SRCS csrc/src/core/plan.cpp csrc/src/core/geometry.cpp csrc/src/core/config.cpp tools/flowbench.cpp; do
  o=build/fb/$(basename $s).o
  objs+=($o)
  if [ ! -f $o ] || [ $s -nt $o ] || [ csrc/src/hip/wave_runner.hpp -nt $o ] || [ csrc/include/gol/hip_kernels.hpp -nt $o ] || [ csrc/include/gol/plan.hpp -nt $o ]; then
    ( hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/include -Wno-unused-result -Wno-unused-value -DGOL_FLOW_EXPERIMENTS $FLAGS -x hip -c $s -o $o || echo "FAILED $s" ) &
  fi
done
wait
hipcc --offload-arch=gfx950 -O3 "${objs[@]}" -o build/flowbench && echo built build/flowbench

#!/bin/bash
# GPU: step_flow against step_temporal passes (tools/flowbench.cpp), 32768^2, several superstep cuts.
# Usage: tools/flow_sweep.sh [out=gpurun_out/flow_sweep.txt] [cut:per_round ...]
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/flow_sweep.txt}
shift
mkdir -p "$(dirname "$out")"
specs=("$@")
[ ${#specs[@]} -eq 0 ] && specs=("8,8,4:1.0" "7,7,6:1.0" "8,8,4:0.67" "8,8,4:1.5" "8,8,8,8,8,8,8,8,8,8,8,8,8,8,8,8:1.0")
for s in "${specs[@]}"; do
  cut=${s%%:*}; pr=${s#*:}
  echo "== cut $cut items/round $pr" | tee -a "$out"
  timeout -k 10 120 build/flowbench 32768 "$cut" 20 "$pr" >> "$out" 2>&1 || { echo "FAILED rc=$? ($s)" | tee -a "$out"; exit 1; }
done

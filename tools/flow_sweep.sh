#!/bin/bash
# GPU: step_flow against step_temporal passes (tools/flowbench.cpp), 32768^2, several superstep cuts.
# Usage: tools/flow_sweep.sh [out=gpurun_out/flow_sweep.txt] [cut:items_per_round:blocks_per_cu:prefetch:last_pass_items_per_round ...]
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/flow_sweep.txt}
shift
mkdir -p "$(dirname "$out")"
specs=("$@")
[ ${#specs[@]} -eq 0 ] && specs=("8,8,4:1.0:0:0" "7,7,6:1.0:0:0" "8,8,4:1.0:0:1" "7,7,6:1.0:0:1" "8,8,4:0.67:0:0"
                                  "8,8,4:1.5:0:0" "7,7,6:1.0:2:0" "8,8,8,8,8,8,8,8,8,8,8,8,8,8,8,8:1.0:0:0"
                                  "8,8,8,8,8,8,8,8,8,8,8,8,8,8,8,8:1.0:0:1" "7,7,6:1.0:0:0:2.0" "8,8,4:1.0:0:0:2.0")
for s in "${specs[@]}"; do
  IFS=: read -r cut pr bpc pf lpr <<< "$s"
  echo "== cut $cut items/round $pr (last pass ${lpr:-$pr}) blocks/CU ${bpc:-auto} prefetch ${pf:-0}" | tee -a "$out"
  KB_FLOW_PF=${pf:-0} KB_LAST_PR=${lpr:-$pr} timeout -k 10 120 build/flowbench 32768 "$cut" 20 "$pr" "${bpc:-0}" >> "$out" 2>&1 || { echo "FAILED rc=$? ($s)" | tee -a "$out"; exit 1; }
done

#!/bin/bash
# with the row-major plan order: XCD permutation on/off (kbench), sub-tile plan occupancy 2 vs 3 (bench, alternating)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2ab
for a in "32768 8 320" "32768 4 160" "32768 1 40" "16384 8 320"; do for s2 in 0 1; do for x in 8 1; do
  r=$(KB_XCDS=$x KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_po $a 2>&1 | tail -1) || exit 1
  echo "xcds=$x split2=$s2 $a $r" | tee -a gpurun_out/r2ab/xcds.txt | sed 's/"skew.*"us_per_gen"/us_per_gen/' | cut -c1-110
done; done; done
for x in 8 1; do r=$(KB_XCDS=$x timeout -k 5 60 ./build/kbench_po 8192 24 960 0 0 8 0 4 2>&1 | tail -1) || exit 1; echo "xcds=$x tile8192 $r" | tee -a gpurun_out/r2ab/xcds.txt | sed 's/"skew.*"us_per_gen"/us_per_gen/' | cut -c1-110; done
for i in 1 2; do for occ in 2 3; do
  GOL_SUB_OCC=$occ timeout -k 10 150 python bench.py --gpus 1 --steps 2000 --warmup 200 > gpurun_out/r2ab/occ$occ_$i.log 2>&1 || exit 1
  echo "sub_occ=$occ 2000 steps: $(tail -1 gpurun_out/r2ab/occ$occ_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("%.3f us/gen" % (d["ms_per_step"]*1e3))')"
  GOL_SUB_OCC=$occ timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2ab/occ20_$occ_$i.log 2>&1 || exit 1
  echo "sub_occ=$occ 20 steps: $(tail -1 gpurun_out/r2ab/occ20_$occ_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("%.3f us/gen" % (d["ms_per_step"]*1e3))')"
done; done

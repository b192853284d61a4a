#!/bin/bash
# small tiles, two workgroups per CU (staging of one overlaps the other's compute): kbench sweep at 8192^2 and 4096x32768
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2t
for shape in "8192 8192" "4096 32768"; do set -- $shape; N=$1; W=$2
for cfg in "24 8 0 4 0" "8 4 34 2 1" "8 4 34 4 1" "12 4 34 2 1" "16 4 34 2 1" "8 8 34 2 1" "8 4 34 2 0" "8 4 34 4 0" "12 4 34 4 0" "16 4 34 4 0" "8 4 23 4 0" "12 4 23 4 0" "16 8 34 4 0" "16 4 45 4 0" "24 4 45 4 1"; do
  set -- $cfg; K=$1; nw=$2; rows=$3; lv=$4; ip=$5
  r=$(KB_W=$W KB_INPLACE=$ip timeout -k 5 60 ./build/kbench_tl $N $K $((K*40)) 0 0 $nw $rows $lv 2>&1 | tail -1) || exit 1
  echo "N=$N W=$W K=$K nw=$nw rows=$rows lv=$lv ip=$ip $r" | tee -a gpurun_out/r2t/sweep.txt | sed 's/"skew.*"rows"/rows/' | cut -c1-175
done; done

#!/bin/bash
# private trash words for non-storing lanes (tr) vs the shared trash row (base = HEAD), 32768^2 and 8192^2 tile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2v
for K in 1 2 4 8; do for s2 in 0 1; do for v in base tr; do
  r=$(KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_$v 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
  echo "$v K=$K split2=$s2 $r" | tee -a gpurun_out/r2v/ab.txt | sed 's/"skew.*"rows"/rows/' | cut -c1-140
done; done; done
for v in base tr; do for args in "8192 24 960 0 0 8 0 4" "4096 32 960 0 0 8 0 2"; do
  r=$(KB_W=$([ "${args%% *}" = 4096 ] && echo 32768 || echo 8192) KB_INPLACE=$([ "${args%% *}" = 4096 ] && echo 1 || echo 0) timeout -k 5 60 ./build/kbench_$v $args 2>&1 | tail -1) || exit 1
  echo "$v tile $args $r" | tee -a gpurun_out/r2v/ab.txt | sed 's/"skew.*"rows"/rows/' | cut -c1-150
done; done

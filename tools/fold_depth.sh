#!/bin/bash
# Folded tiles at 8192^2: pass depth 32 vs 40 / 48 / 64 (kbench, alternating, 8 waves, 4 levels per LDS pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fold
for rep in 1 2 3; do for k in 32 40 48 64; do
  echo "fold K=$k $(KB_FOLD=1 timeout -k 5 60 build/kbench_main 8192 $k 1920 0 0 8 0 4 | grep -o '"rows": [0-9]*\|"us_per_gen": [0-9.]*' | tr '\n' ' ')" || exit 1
done; done | tee gpurun_out/fold/fold_depth.txt

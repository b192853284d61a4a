#!/bin/bash
# The 4096 x 32768 per-rank strip (config 3 strong-scaled over 8 GPUs): folded tiles at depths whose
# plan fits one round (K <= 15) vs the in-place tile kernel, alternating (kbench, KB_W=32768).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fold
K() { timeout -k 5 60 build/kbench_main "$@"; }
{
echo "check fold K=12"; KB_CHECK=1 KB_FOLD=1 KB_W=32768 K 4096 12 960 0 0 8 0 4 || exit $?
for rep in 1 2; do
  for k in 8 12 15; do
    echo "fold K=$k"; KB_FOLD=1 KB_W=32768 K 4096 $k 960 0 0 8 0 4 || exit $?
  done
  for k in 16 24; do
    echo "base-inplace K=$k"; KB_INPLACE=1 KB_W=32768 K 4096 $k 960 0 0 8 0 2 || exit $?
  done
done
} 2>&1 | tee gpurun_out/fold/fold_strip.txt

#!/bin/bash
# The 4096 x 32768 per-rank strip (config 3 strong-scaled over 8 GPUs): folded in-place tiles (one
# round) vs the in-place tile kernel, alternating (kbench, KB_W=32768), with word-by-word checks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fold
K() { timeout -k 5 60 build/kbench_main "$@"; }
{
for cfg in "4096 24 960 0 0 8 0 2" "4096 13 960 0 0 8 0 4" "2048 7 960 0 0 16 0 2"; do
  echo "check fold-inplace $cfg"; KB_CHECK=1 KB_INPLACE=1 KB_FOLD=1 KB_W=32768 K $cfg || exit $?
done
for rep in 1 2; do
  for k in 16 24 32; do
    for lv in 2 4; do
      echo "fold-inplace K=$k lv=$lv"; KB_INPLACE=1 KB_FOLD=1 KB_W=32768 K 4096 $k 960 0 0 8 0 $lv || exit $?
    done
    echo "base-inplace K=$k lv=2"; KB_INPLACE=1 KB_W=32768 K 4096 $k 960 0 0 8 0 2 || exit $?
  done
done
} 2>&1 | tee gpurun_out/fold/fold_strip.txt

#!/bin/bash
# Folded tile kernel (STEP_TILE_FOLD) vs the tile kernel: correctness (KB_CHECK=1: K generations vs K
# single-generation temporal passes, every word) and alternating timing at 8192^2 and the 4096 x 32768
# strip of config 3 strong-scaled over 8 GPUs.  kbench args: N K gens pf skew nw rows lv.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fold
export TMPDIR=/tmp
K() { timeout -k 5 60 build/kbench_main "$@"; }
set -o pipefail
{
echo "## correctness"
for cfg in "8192 24 960 0 0 8 0 4" "8192 16 960 0 0 8 0 2" "8192 7 960 0 0 4 0 1" "4096 24 960 0 0 8 0 4" "1024 9 960 0 0 8 0 4" "3072 13 960 0 0 8 0 2"; do
  echo "fold $cfg"; KB_CHECK=1 KB_FOLD=1 K $cfg || exit $?
done
echo "base 8192 24 960 0 0 8 0 4"; KB_CHECK=1 K 8192 24 960 0 0 8 0 4 || exit $?
echo "## timing 8192^2 (us/gen)"
for rep in 1 2; do
  for k in 16 24 32; do
    for nw in 8 16; do
      echo "base K=$k nw=$nw"; K 8192 $k 960 0 0 $nw 0 4 || exit $?
      echo "fold K=$k nw=$nw"; KB_FOLD=1 K 8192 $k 960 0 0 $nw 0 4 || exit $?
    done
  done
done
echo "## timing 4096 x 32768 (KB_W=32768)"
for k in 16 24 32; do
  echo "base K=$k"; KB_W=32768 K 4096 $k 960 0 0 8 0 4 || exit $?
  echo "base-inplace K=$k"; KB_INPLACE=1 KB_W=32768 K 4096 $k 960 0 0 8 0 4 || exit $?
  echo "fold K=$k"; KB_FOLD=1 KB_W=32768 K 4096 $k 960 0 0 8 0 4 || exit $?
done
} 2>&1 | tee gpurun_out/fold/fold_ab.txt

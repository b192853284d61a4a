#!/bin/bash
# Tile kernel band loop: two register triples (GOL_TILE_PINGPONG=1) vs one, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2be
mkdir -p $o
: > $o/ab.txt
run() {  # run <label> <env...> -- <kbench args>
  local label=$1; shift
  for bin in tbase tpp; do
    r=$(env "$@" timeout -k 5 60 ./build/kbench_$bin $KBARGS 2>&1 | tail -1) || return 1
    echo "$bin $label $r" | sed 's/"skew.*"tile_nw"/tile_nw/' | tee -a $o/ab.txt
  done
}
for rep in 1 2; do
  KBARGS="8192 24 960 0 0 8 0 4" run "8192 K24 lv4 db" KB_INPLACE=0 || exit 1
  KBARGS="8192 16 960 0 0 8 0 2" run "8192 K16 lv2 db" KB_INPLACE=0 || exit 1
  KBARGS="4096 16 640 0 0 8 0 2" run "4096x32768 K16 lv2 ip" KB_W=32768 KB_INPLACE=1 || exit 1
  KBARGS="16384 16 640 0 0 8 0 2" run "16384 K16 lv2 ip" KB_INPLACE=1 || exit 1
done

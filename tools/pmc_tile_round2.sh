#!/bin/bash
# PMC of the round-2 tile kernel at its auto configuration for 8192^2 (K=24, 8 waves, 4 generations
# per LDS pass, double-buffered), for comparison with the round-1 PMC (K=16, 2 per LDS pass).
# One counter set per run, --kernel-trace only.  Output: gpurun_out/pmc_tile_r2/*.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/pmc_tile_r2
mkdir -p $o
pmc() {  # pmc <name> <counters> -- <kbench args>
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $ctr -d $o/$name -o $name --output-format csv -- $R/build/kbench_main "$@" > $o/$name.log 2>&1 || { echo "$name failed"; return 1; }
  echo "$name ok"
}
pmc tile_a "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" 8192 24 480 0 0 8 0 4 &&
pmc tile_b "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" 8192 24 480 0 0 8 0 4 &&
pmc tile_old_a "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" 8192 16 480 0 0 8 0 2 &&
pmc tile_old_b "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" 8192 16 480 0 0 8 0 2 &&
for n in tile_a tile_b tile_old_a tile_old_b; do
  f=$(find $o/$n -name '*counter_collection.csv' | head -1)
  echo "== $n"; python3 $R/tools/pmc_summary.py "$f"
done > $o/summary.txt

#!/bin/bash
# PMC counters of the hot kernels (kbench, 32768^2: temporal K=8; 8192^2: tile K=16).  Counter runs
# use --kernel-trace only (no sys/runtime traces).  Output: gpurun_out/pmc_temporal/*.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/pmc_temporal
mkdir -p $o
pmc() {  # pmc <name> <counters> -- <kbench args>
  local name=$1 ctr=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d $o/$name -o $name --output-format csv -- $R/build/kbench_tile "$@" > $o/$name.log 2>&1
  echo "$name rc=$?"
}
pmc t_a "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" 32768 8 240 0 0 0
pmc t_b "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" 32768 8 240 0 0 0
pmc t_c "FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE" 32768 8 240 0 0 0
pmc tile_a "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" 8192 16 480 0 0 8 0 2
pmc tile_c "FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE" 8192 16 480 0 0 8 0 2

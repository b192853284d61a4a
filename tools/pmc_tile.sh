cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_tile
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/pmc_tile/a -o a --output-format csv -- $R/build/kbench_tile 32768 8 480 0 0 16 > $R/gpurun_out/pmc_tile/a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES -d $R/gpurun_out/pmc_tile/b -o b --output-format csv -- $R/build/kbench_tile 32768 8 480 0 0 16 > $R/gpurun_out/pmc_tile/b.log 2>&1 || exit $?

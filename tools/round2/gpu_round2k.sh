#!/bin/bash
# shallow-pass prefetch depth A/B (kbench, 32768^2) + engine bench + tile-kernel PMC at 8192^2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2k
export TMPDIR=/tmp
for K in 1 2 3 4; do
  for bpc in 3 8; do
    for s2 in 0 1; do
      for v in pf0 pf1; do
        r=$(KB_BPC=$bpc KB_SPLIT2=$s2 timeout -k 5 60 ./build/kbench_$v 32768 $K $((K*40)) 2>&1 | tail -1) || exit 1
        echo "$v K=$K bpc=$bpc split2=$s2 $r" | tee -a gpurun_out/r2k/pf_sweep.txt
      done
    done
  done
done
for i in 1 2 3; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2k/bench_$i.log 2>&1 || exit 1; tail -1 gpurun_out/r2k/bench_$i.log | cut -c1-330; done
timeout -k 10 120 python bench.py --gpus 1 --steps 2000 --warmup 200 > gpurun_out/r2k/bench_long.log 2>&1 || exit 1; tail -1 gpurun_out/r2k/bench_long.log | cut -c1-330
cd /tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/r2k/pmc_a -o a --output-format csv -- $R/build/kbench_pf1 8192 24 960 0 0 8 0 2 > $R/gpurun_out/r2k/pmc_a.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES -d $R/gpurun_out/r2k/pmc_b -o b --output-format csv -- $R/build/kbench_pf1 8192 24 960 0 0 8 0 2 > $R/gpurun_out/r2k/pmc_b.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM SQ_WAVE32_INSTS GRBM_GUI_ACTIVE SQ_IFETCH SQ_INSTS_BRANCH -d $R/gpurun_out/r2k/pmc_c -o c --output-format csv -- $R/build/kbench_pf1 8192 24 960 0 0 8 0 2 > $R/gpurun_out/r2k/pmc_c.log 2>&1 || echo "pmc_c failed (optional)"
echo done

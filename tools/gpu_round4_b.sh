#!/bin/bash
# GPU batch B (round 4): BASELINE configs on the final tree, the 8-process torchrun rehearsal (per-rank
# arrays), self-exchange runs (RCCL registered / unregistered, flow+ov), and PMC counters of the flow
# kernel vs the pass kernel.  Each step has its own time limit; a fatal status ends the batch.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "[batch-b] $(date +%T) $*"; }
step configs
bash tools/baseline_configs.sh cfg2 cfg2f cfg2nf cfg2 cfg2f cfg2nf cfg2b cfg3 cfg4 > gpurun_out/configs_summary.txt 2>&1 || { cat gpurun_out/configs_summary.txt; exit 1; }
step self-exchange
for v in "GOL_RCCL_REGISTER=1" "GOL_RCCL_REGISTER=0" "GOL_SCHEDULE=flow+ov" "GOL_SCHEDULE=flow"; do
  env $v timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange > gpurun_out/selfx_$(echo $v | tr '=+' '__').json 2> gpurun_out/selfx_err.txt || { echo "self-exchange $v failed"; tail gpurun_out/selfx_err.txt; exit 1; }
done
step rehearsal
timeout -k 10 900 bash tools/rehearse_torchrun.sh > gpurun_out/rehearse_summary.txt 2>&1 || { tail -30 gpurun_out/rehearse_summary.txt; exit 1; }
step pmc
for kn in flow temporal; do
  if [ $kn = flow ]; then envs="GOL_SCHEDULE=flow"; else envs="GOL_SUBTILES=0"; fi
  env $envs timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d gpurun_out/pmc_$kn -o pmc -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-phases > gpurun_out/pmc_$kn.txt 2>&1 || { echo "pmc $kn rc=$?"; tail gpurun_out/pmc_$kn.txt; exit 1; }
done
step done

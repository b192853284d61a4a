#!/bin/bash
# GPU batch D (round 4): the full GPU test suite and smoke on the current tree, the driver's bench
# command x5 (headline), the 8-process rehearsal (strong / 2-D after the per-rank kernel fix), and
# PMC of config 2 (tile passes vs tile flow).  Each step has its own time limit; stops at a failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
s() { echo "[batch-d] $(date +%T) $*"; }
s tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
s smoke
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail gpurun_out/smoke.log; exit 1; }
s driver-bench
: > gpurun_out/driver_bench.jsonl
for i in 1 2 3 4 5; do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/driver_bench.jsonl 2>gpurun_out/driver_bench.err || { echo "bench rc=$?"; tail gpurun_out/driver_bench.err; exit 1; }
done
python3 -c "
import json
for l in open('gpurun_out/driver_bench.jsonl'):
    d=json.loads(l); print('%.3f us/gen' % (d['ms_per_step']*1e3), d['config']['schedule'], d['config']['kernel'])
"
s rehearsal
timeout -k 10 900 bash tools/rehearse_torchrun.sh > gpurun_out/rehearse_summary.txt 2>&1 || { tail -30 gpurun_out/rehearse_summary.txt; exit 1; }
grep -E "^==|rc=|value" gpurun_out/rehearse_summary.txt
s pmc
for kn in flow tile; do
  if [ $kn = flow ]; then envs="GOL_SCHEDULE=flow"; else envs="GOL_SCHEDULE=auto"; fi
  env $envs timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d gpurun_out/pmc_cfg2_$kn -o pmc -- ./build/gol 5 8192 1000 256 0 > gpurun_out/pmc_cfg2_$kn.txt 2>&1 || { echo "pmc $kn rc=$?"; tail gpurun_out/pmc_cfg2_$kn.txt; exit 1; }
done
s done

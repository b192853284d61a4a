#!/bin/bash
# GPU (round 4, final tree): the full GPU suite and smoke, the driver's bench command x3 and its cut
# through the RCCL self-exchange x3.  Each step has its own time limit; stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
s() { echo "[final] $(date +%T) $*"; }
s tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_final.log
s smoke
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { echo "smoke rc=$?"; tail gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
s bench
o=gpurun_out/final_bench.txt
: > $o
for v in "" "--self-exchange"; do
  for i in 1 2 3; do
    r=$(timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 $v 2>/dev/null) || { echo "bench rc=$? ($v)"; exit 1; }
    echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('[$v] %.3f us/gen' % (d['ms_per_step']*1e3), '%.4g' % d['value'], c['schedule'], c['kernel'])" | tee -a $o || exit 1
  done
done
s done

#!/bin/bash
# GPU: the sub-tile overlap tests, then the driver's cut through the RCCL self-exchange x4 and one trace.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py -x -q --timeout 180 --timeout-method thread -k "subtile or overlap or self" > gpurun_out/test_subtiles.txt 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/test_subtiles.txt; exit 1; }
tail -2 gpurun_out/test_subtiles.txt
o=gpurun_out/selfx_round4b.txt
: > $o
for i in 1 2 3 4; do
  r=$(timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange 2>/dev/null) || { echo "selfx rc=$?"; exit 1; }
  echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; p=d['phases']; print('self-exchange: %.3f us/gen' % (d['ms_per_step']*1e3), c['schedule'], c['kernel'], 'exchange_us', p.get('exchange_us_max'), 'superstep_us', p.get('superstep_us_max'), [x for x in c['autotune'].split() if x.startswith('sched:')])" | tee -a $o || exit 1
done
bash tools/gpu_trace_selfx.sh

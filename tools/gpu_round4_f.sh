#!/bin/bash
# GPU batch F (round 4): the driver command against the round-3 tree after the K=12 fix, and the
# driver's cut through the RCCL self-exchange x3.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash tools/gpu_ab_tree.sh build/r3src 5 || exit 1
o=gpurun_out/selfx_round4.txt
: > $o
for i in 1 2 3; do
  r=$(timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange 2>/dev/null) || { echo "selfx rc=$?"; exit 1; }
  echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; p=d['phases']; print('self-exchange: %.3f us/gen' % (d['ms_per_step']*1e3), c['schedule'], c['kernel'], 'registered', c['rccl_registered'], 'exchange_us', p.get('exchange_us_max'), 'superstep_us', p.get('superstep_us_max'))" | tee -a $o || exit 1
done

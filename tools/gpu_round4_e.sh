#!/bin/bash
# GPU batch E (round 4): the 8192^2 warmup anomaly against the XCD-aware plan order (GOL_PLAN_XCDS=8 / 1,
# warmups 96 / 100), config 2 with the flow candidates timed (GOL_FLOW=1: equal-span timing), and the
# driver's cut through the RCCL self-exchange x3.  Each step has its own time limit.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/warmup_xcds.txt
: > $o
for round in 1 2; do
  for x in 8 1; do
    for w in 96 100; do
      r=$(GOL_PLAN_XCDS=$x timeout -k 10 120 python3 bench.py --size 8192 --steps 1000 --warmup $w --no-phases 2>/dev/null) || { echo "bench rc=$? (xcds $x warmup $w)"; exit 1; }
      echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('xcds $x warmup $w: %.4f us/gen' % (d['ms_per_step']*1e3), d['config']['schedule'], d['config']['kernel'])" | tee -a $o
    done
  done
done
for i in 1 2; do
  echo "== cfg2 CLI GOL_FLOW=1" | tee -a $o
  GOL_BACKEND=hip GOL_FLOW=1 GOL_METRICS_JSON=gpurun_out/cfg2_flowtimed.json timeout -k 10 120 ./build/gol 5 8192 1000 256 0 > gpurun_out/cfg2_flowtimed.log 2>&1 || { echo "cli rc=$?"; tail gpurun_out/cfg2_flowtimed.log; exit 1; }
  grep -E "TOTAL" gpurun_out/cfg2_flowtimed.log | tee -a $o
  python3 -c "import json; d=json.load(open('gpurun_out/cfg2_flowtimed.json')); s=json.dumps(d); import re; print(re.findall(r'\"schedule\": \"[^\"]*\"', s)[:1], re.findall(r'sched:[a-z+]*=[0-9.]*', s))" | tee -a $o
done
for i in 1 2 3; do
  r=$(timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange 2>/dev/null) || { echo "selfx rc=$?"; exit 1; }
  echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; p=d['phases']; print('self-exchange: %.3f us/gen' % (d['ms_per_step']*1e3), c['schedule'], c['kernel'], 'registered', c['rccl_registered'], 'exchange_us', p.get('exchange_us_max'), 'superstep_us', p.get('superstep_us_max'))" | tee -a $o
done

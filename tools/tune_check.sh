#!/bin/bash
# bench.py three times at 32768^2 and once at 16384^2 / 8192^2: autotune picks and their stability.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune
for n in 32768 32768 32768 16384 8192; do
  timeout -k 10 120 python bench.py --size $n --steps 2000 --warmup 200 >> gpurun_out/tune/b.log 2>&1 || exit 3
done
grep '^{' gpurun_out/tune/b.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); c=d['config']; print(c['board'][0], round(d['ms_per_step']*1e3,3), c['kernel'], c['kernel_depth'], c['autotune'][:150])"

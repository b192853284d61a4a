#!/bin/bash
# Two sub-tiles: 64- vs 128-generation supersteps (the streams meet once per superstep), alternating.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sub
out=gpurun_out/sub/r128.txt; : > $out
for r in 1 2 3; do
  for hd in 64 128; do
    GOL_HALO_DEPTH=$hd timeout -k 10 150 python bench.py --size 32768 --steps 2048 --warmup 128 > gpurun_out/sub/b.log 2>&1 || { tail -5 gpurun_out/sub/b.log; exit 3; }
    grep '^{' gpurun_out/sub/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('R=$hd', c['board'][0], round(d['ms_per_step']*1e3,3), 'us/gen', '%.3e' % d['value'], c['schedule'])" >> $out
  done
done
cat $out

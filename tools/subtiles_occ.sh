#!/bin/bash
# Two sub-tiles: halves planned for 2 waves/SIMD (default) vs the single-tile tuned occupancy, alternating.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sub
out=gpurun_out/sub/occ.txt; : > $out
for r in 1 2 3; do
  for so in 2 3; do
    GOL_SUB_OCC=$so timeout -k 10 150 python bench.py --size 32768 --steps 2048 --warmup 128 > gpurun_out/sub/b.log 2>&1 || { tail -5 gpurun_out/sub/b.log; exit 3; }
    grep '^{' gpurun_out/sub/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('sub_occ=$so', c['board'][0], round(d['ms_per_step']*1e3,3), 'us/gen', '%.3e' % d['value'], c['schedule'])" >> $out
  done
done
for so in 2 3; do
  GOL_SUB_OCC=$so timeout -k 10 150 python bench.py --size 65536 --steps 256 --warmup 32 > gpurun_out/sub/b.log 2>&1 || exit 3
  grep '^{' gpurun_out/sub/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('sub_occ=$so', c['board'][0], round(d['ms_per_step']*1e3,3), 'us/gen', '%.3e' % d['value'], c['schedule'])" >> $out
done
cat $out

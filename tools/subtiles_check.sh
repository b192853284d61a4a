#!/bin/bash
# GOL_SUBTILES=2 (two half-tiles per rank on two streams) vs one tile: bench.py at 32768^2 / 16384^2,
# halo depth 32 and 64, alternating.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sub
out=gpurun_out/sub/bench.txt; : > $out
for r in 1 2; do
  for n in 32768 16384; do
    for cfg in 0:0 2:0 2:64; do
      sub=${cfg%%:*}; hd=${cfg#*:}
      GOL_SUBTILES=$sub GOL_HALO_DEPTH=$hd timeout -k 10 150 python bench.py --size $n --steps 2048 --warmup 128 > gpurun_out/sub/b.log 2>&1 || { tail -5 gpurun_out/sub/b.log; exit 3; }
      grep '^{' gpurun_out/sub/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('sub=$sub R=$hd', c['board'][0], round(d['ms_per_step']*1e3,3), 'us/gen', '%.3e' % d['value'], c['kernel'], c['schedule'])" >> $out
    done
  done
done
cat $out

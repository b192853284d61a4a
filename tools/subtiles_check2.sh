#!/bin/bash
# GOL_SUBTILES=2 at 65536^2 and 32768^2 (R=64) vs one tile, and thread ranks (1-D P=2) with sub-tiles.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sub
out=gpurun_out/sub/bench2.txt; : > $out
for r in 1 2; do
  for cfg in 65536:0:0 65536:2:64 32768:0:0 32768:2:64; do
    IFS=: read n sub hd <<< "$cfg"
    st=1024; [ $n = 65536 ] && st=256
    GOL_SUBTILES=$sub GOL_HALO_DEPTH=$hd timeout -k 10 150 python bench.py --size $n --steps $st --warmup 64 > gpurun_out/sub/b.log 2>&1 || { tail -5 gpurun_out/sub/b.log; exit 3; }
    grep '^{' gpurun_out/sub/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('sub=$sub R=$hd', c['board'][0], round(d['ms_per_step']*1e3,3), 'us/gen', '%.3e' % d['value'], c['schedule'])" >> $out
  done
done
for sub in 0 2; do
  GOL_SUBTILES=$sub GOL_SCHEDULE=full timeout -k 10 200 python -u tools/rehearse_multirank.py --configs 1d:2:32768 --gens 2560 | sed "s/^/sub=$sub /" >> $out || exit 3
done
cat $out

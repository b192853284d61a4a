#!/bin/bash
# Config-2 sweep of bench.py at 8192^2: kernel:halo-depth:kernel-depth specs (auto vs fixed tile depths).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg2
for spec in "auto:16:0" "tile:16:16" "tile:32:32" "tile:32:16" "tile:24:24"; do
  IFS=: read kern R K <<< "$spec"
  timeout -k 10 120 python bench.py --size 8192 --steps 2000 --warmup 200 --kernel $kern --halo-depth $R --kernel-depth $K > gpurun_out/cfg2/$kern-$R-$K.log 2>&1 || { echo "$spec failed"; tail -3 gpurun_out/cfg2/$kern-$R-$K.log; continue; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/cfg2/$kern-$R-$K.log') if l.startswith('{')][-1]); c=d['config']; print('$spec %.4e %.3f us/gen kernel=%s K=%s waves=%s %s' % (d['value'], d['ms_per_step']*1e3, c['kernel'], c['kernel_depth'], c['tile_waves'], c['autotune'][:100]))"
done

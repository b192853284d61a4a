#!/bin/bash
# bench.py at 8192^2 / 16384^2 / 32768^2 (autotune strings show the 3- vs 2-waves/SIMD temporal plans) and the
# one-GPU multi-rank rehearsal at strong-scaling tile sizes.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/occ
for n in 8192 16384 32768; do
  timeout -k 10 120 python bench.py --size $n --steps 2000 --warmup 200 > gpurun_out/occ/b$n.log 2>&1 || exit 3
done
timeout -k 10 300 python -u tools/rehearse_multirank.py --configs 1d:8:32768,1d:4:32768 > gpurun_out/occ/rm.txt 2>&1 || exit 3
for f in gpurun_out/occ/b*.log; do grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$f', round(d['ms_per_step']*1e3,3), c['kernel'], c['kernel_depth'], c['autotune'])"; done
cat gpurun_out/occ/rm.txt

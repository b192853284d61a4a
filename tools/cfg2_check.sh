#!/bin/bash
# BASELINE config 2 on one GPU: bench.py at 8192^2 and the reference CLI (8192^2 x 1000).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg2
timeout -k 10 120 python bench.py --size 8192 --steps 2000 --warmup 200 > gpurun_out/cfg2/bench8192.log 2>&1 || exit 3
for i in 1 2 3; do timeout -k 10 120 ./build/gol 5 8192 1000 256 0 >> gpurun_out/cfg2/cli8192.log 2>&1 || exit 3; done
grep '^{' gpurun_out/cfg2/bench8192.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('bench8192', round(d['ms_per_step']*1e3,3), 'us/gen', c['kernel'], c['kernel_depth'], c['halo_depth'], c['graph_launches'])"
grep TOTAL gpurun_out/cfg2/cli8192.log

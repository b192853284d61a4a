#!/bin/bash
# Driver command with GOL_SYNC_SPIN=0 (hipStreamSynchronize) vs 1 (busy-poll hipStreamQuery first), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/spin
for i in 1 2 3 4; do for v in 0 1; do
  GOL_SYNC_SPIN=$v timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/spin/b_$v_$i.log 2>&1 || exit 3
  grep '^{' gpurun_out/spin/b_$v_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('spin=$v', round(d['ms_per_step']*1e3,3), 'us/gen')"
done; done | tee gpurun_out/spin/ab.txt

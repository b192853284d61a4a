#!/bin/bash
# Folded tiles in the engine: GPU suite, config 2 (bench + CLI) with GOL_TILE_FOLD auto (=on) vs 0,
# alternating, and the driver command (unchanged path) for regressions.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/foldeng
export TMPDIR=/tmp
o=gpurun_out/foldeng
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $o/pytest.log 2>&1; rc=$?
tail -3 $o/pytest.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for f in -1 0; do
    GOL_TILE_FOLD=$f timeout -k 10 120 python bench.py --size 8192 --steps 2000 --warmup 200 > $o/b8192_$f.log 2>&1 || exit 3
    grep '^{' $o/b8192_$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('fold=$f bench8192', round(d['ms_per_step']*1e3,3), 'us/gen', '%.3e' % d['value'], c['kernel'], c['kernel_depth'], c['halo_depth'], c['autotune'])"
    for i in 1 2; do GOL_TILE_FOLD=$f timeout -k 10 120 ./build/gol 5 8192 1000 256 0 > $o/cli_$f.log 2>&1 || exit 3; echo "fold=$f cli $(grep TOTAL $o/cli_$f.log)"; done
  done
done
for i in 1 2 3; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/drv$i.log 2>&1 || exit 3
  grep '^{' $o/drv$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('driver', round(d['ms_per_step']*1e3,3), 'us/gen', '%.3e' % d['value'], d['config']['schedule'])"; done

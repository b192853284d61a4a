#!/bin/bash
# Asynchronous sub-tile superstep starts (GOL_SUBTILE_ASYNC): sub-tile GPU tests, headline oracle, then
# alternating benches (20, 256, 2000 steps) with and without.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2aw
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_headline.py tests/test_gpu_rccl.py -k "subtile or headline or run_hint or rccl" -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for rep in 1 2; do
  for steps in 20 256 2000; do
    for as in 0 1; do
      timeout -k 10 120 env GOL_SUBTILE_ASYNC=$as python bench.py --gpus 1 --steps $steps --warmup 5 > $o/a${as}_${steps}_$rep.log 2>&1 || exit 1
      grep '^{"metric"' $o/a${as}_${steps}_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); print("async '$as' steps '$steps': %.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]), d["config"]["schedule"])'
    done
  done
done

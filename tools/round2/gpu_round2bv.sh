#!/bin/bash
# Sub-tile cross-stream signals in signal memory (GOL_SUB_SYNC=value, default) vs events: tests, then alternating benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2bv
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py tests/test_gpu_headline.py -k "subtile or rccl or headline or run_hint or checkpoint" -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for rep in 1 2 3; do
  for sy in event value; do
    for cfg in "self20 --steps 20 --warmup 5 --self-exchange" "loc20 --steps 20 --warmup 5" "loc2k --steps 2048 --warmup 128"; do
      set -- $cfg; n=$1; shift
      timeout -k 10 150 env GOL_SUB_SYNC=$sy python bench.py --gpus 1 "$@" > $o/${n}_${sy}_$rep.log 2>&1 || { tail -3 $o/${n}_${sy}_$rep.log; exit 1; }
      grep '^{"metric"' $o/${n}_${sy}_$rep.log | python -c 'import json,sys; d=json.load(sys.stdin); print("'$n' '$sy' %.3f us/gen" % (d["ms_per_step"]*1e3))'
    done
  done
done

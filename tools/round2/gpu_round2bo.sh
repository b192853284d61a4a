#!/bin/bash
# Auto halo depth 128 for 1-D strips with neighbours: GPU engine + RCCL tests, per-rank tiles through self-exchange.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2bo
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py tests/test_gpu_cli.py -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
b() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 150 python bench.py --gpus 1 "$@" > $o/$n.log 2>&1 || { echo "$n failed"; tail -5 $o/$n.log; exit 1; }
  echo "$n $(grep '^{"metric"' $o/$n.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("%.3e" % d["value"], "%.3f us/gen" % (d["ms_per_step"]*1e3), c["tile_per_rank"], c["schedule"], c["kernel"], "R=%s K=%s" % (c["halo_depth"], c["kernel_depth"]), c["transport"], [x for x in c["autotune"].split() if x.startswith("sched")])')"
}
b s3_self --steps 1280 --warmup 128 --size 4096 --width 32768 --self-exchange
b s2_self --steps 1280 --warmup 128 --size 16384 --width 32768 --self-exchange
b c4_2d_self --steps 1120 --warmup 112 --size 32768 --width 16384 --decomp 2d --self-exchange
b c4_1d_self --steps 1280 --warmup 128 --size 8192 --width 65536 --self-exchange

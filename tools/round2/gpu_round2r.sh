#!/bin/bash
# tile variant per plan (double-buffered when one round fits, else in place): tests + configs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2r
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_cli.py -x -q -m gpu -k "tile or auto or cfg or perf" --timeout 120 --timeout-method thread > gpurun_out/r2r/pytest.log 2>&1 || { tail -30 gpurun_out/r2r/pytest.log; exit 1; }
tail -1 gpurun_out/r2r/pytest.log
for i in 1 2 3; do timeout -k 10 60 ./build/gol 5 8192 1000 256 0 > gpurun_out/r2r/cfg2_$i.txt || exit 1; head -1 gpurun_out/r2r/cfg2_$i.txt; done
b() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 150 python bench.py --gpus 1 "$@" > gpurun_out/r2r/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/r2r/$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/r2r/$n.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("%.3e" % d["value"], "%.3f us/gen" % (d["ms_per_step"]*1e3), c["tile_per_rank"], c["schedule"], c["kernel"], "R=%s K=%s" % (c["halo_depth"], c["kernel_depth"]), c["transport"], c["autotune"][:300])')"
}
b c2 --steps 2000 --warmup 200 --size 8192
b s3_local --steps 1280 --warmup 128 --size 4096 --width 32768
b s3_self --steps 1280 --warmup 128 --size 4096 --width 32768 --self-exchange
b b16k --steps 1000 --warmup 100 --size 16384

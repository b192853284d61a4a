#!/bin/bash
# row-major plan order: full GPU suite, driver bench x3, long bench, BASELINE configs on one GPU
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2aa
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2aa/pytest.log 2>&1 || { tail -30 gpurun_out/r2aa/pytest.log; exit 1; }
tail -1 gpurun_out/r2aa/pytest.log
b() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 150 python bench.py --gpus 1 "$@" > gpurun_out/r2aa/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/r2aa/$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/r2aa/$n.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("%.3e" % d["value"], "%.3f us/gen" % (d["ms_per_step"]*1e3), c["tile_per_rank"], c["schedule"], c["kernel"], "R=%s K=%s" % (c["halo_depth"], c["kernel_depth"]), c["transport"])')"
}
for i in 1 2 3 4 5; do b bench20_$i --steps 20 --warmup 5; done
b bench2000 --steps 2000 --warmup 200
b c2 --steps 2000 --warmup 200 --size 8192
b b16k --steps 1000 --warmup 100 --size 16384
b s3_self --steps 1280 --warmup 128 --size 4096 --width 32768 --self-exchange
b c4_2d_self --steps 1120 --warmup 112 --size 32768 --width 16384 --decomp 2d --self-exchange
b w_self --steps 1280 --warmup 128 --self-exchange
b b65k --steps 256 --warmup 32 --size 65536
for i in 1 2 3; do timeout -k 10 60 ./build/gol 5 8192 1000 256 0 > gpurun_out/r2aa/cfg2_$i.txt || exit 1; head -1 gpurun_out/r2aa/cfg2_$i.txt; done

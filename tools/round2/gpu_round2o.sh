#!/bin/bash
# tile kernel 4-level LDS passes A/B; deeper auto halos + fixed schedule timing on the per-rank tiles; GPU engine tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_rccl.py -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/r2o/pytest.log 2>&1 || { tail -30 gpurun_out/r2o/pytest.log; exit 1; }
tail -1 gpurun_out/r2o/pytest.log
for N in 8192 16384; do for K in 16 24 32; do for nw in 8 16; do for lv in 2 4; do
  r=$(timeout -k 5 60 ./build/kbench_tl $N $K $((K*40)) 0 0 $nw 0 $lv 2>&1 | tail -1) || exit 1
  echo "N=$N K=$K nw=$nw lv=$lv $r" | tee -a gpurun_out/r2o/tile_lv.txt | cut -c1-40,170-
done; done; done; done
b() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 150 python bench.py --gpus 1 "$@" > gpurun_out/r2o/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/r2o/$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/r2o/$n.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("%.3e" % d["value"], "%.3f us/gen" % (d["ms_per_step"]*1e3), c["tile_per_rank"], c["schedule"], c["kernel"], "R=%s K=%s" % (c["halo_depth"], c["kernel_depth"]), c["transport"], [x for x in c["autotune"].split() if x.startswith("sched")])')"
}
b s3_self --steps 1280 --warmup 128 --size 4096 --width 32768 --self-exchange
b c4_2d_self --steps 1120 --warmup 112 --size 32768 --width 16384 --decomp 2d --self-exchange
b c4_1d_self --steps 1280 --warmup 128 --size 8192 --width 65536 --self-exchange
b w_self --steps 1280 --warmup 128 --self-exchange
b bench20 --steps 20 --warmup 5

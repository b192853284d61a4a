#!/bin/bash
# Per-rank tiles of the multi-GPU configs through RCCL self-exchange, after the two-triple loop and the deeper pass costs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2bh
mkdir -p $o
b() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 150 python bench.py --gpus 1 "$@" > $o/$n.log 2>&1 || { echo "$n failed"; tail -5 $o/$n.log; exit 1; }
  echo "$n $(grep '^{"metric"' $o/$n.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("%.3e" % d["value"], "%.3f us/gen" % (d["ms_per_step"]*1e3), c["tile_per_rank"], c["schedule"], c["kernel"], "R=%s K=%s" % (c["halo_depth"], c["kernel_depth"]), c["transport"], [x for x in c["autotune"].split() if x.startswith("sched")])')"
}
b s3_self --steps 1280 --warmup 128 --size 4096 --width 32768 --self-exchange
b c4_2d_self --steps 1120 --warmup 112 --size 32768 --width 16384 --decomp 2d --self-exchange
b c4_1d_self --steps 1280 --warmup 128 --size 8192 --width 65536 --self-exchange
b w_self --steps 1280 --warmup 128 --self-exchange
b w_self20 --steps 20 --warmup 5 --self-exchange
b w_self20b --steps 20 --warmup 5 --self-exchange

#!/bin/bash
# two sub-tiles forced on smaller tiles (below the auto threshold of 24576 rows): 16384^2, 4096 x 32768, 8192^2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2ak
b() {  # name, env, bench args...
  local n=$1 e=$2; shift 2
  env $e timeout -k 10 150 python bench.py --gpus 1 "$@" > gpurun_out/r2ak/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/r2ak/$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/r2ak/$n.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("%.3e" % d["value"], "%.3f us/gen" % (d["ms_per_step"]*1e3), c["schedule"], c["kernel"], "R=%s" % c["halo_depth"], [x for x in c["autotune"].split() if x.startswith("sched")])')"
}
for i in 1 2; do
b b16k_auto_$i GOL_SUBTILES=auto --steps 1024 --warmup 128 --size 16384
b b16k_sub_$i GOL_SUBTILES=2 --steps 1024 --warmup 128 --size 16384
b s3_auto_$i GOL_SUBTILES=auto --steps 1024 --warmup 128 --size 4096 --width 32768
b s3_sub_$i GOL_SUBTILES=2 --steps 1024 --warmup 128 --size 4096 --width 32768
b s3self_sub_$i GOL_SUBTILES=2 --steps 1024 --warmup 128 --size 4096 --width 32768 --self-exchange
b c2_sub_$i GOL_SUBTILES=2 --steps 1024 --warmup 128 --size 8192
done

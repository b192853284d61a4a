#!/bin/bash
# per-rank tiles of the scaling configs on one GPU (rectangular boards, RCCL self-exchange) + 2-D vs 1-D rehearsal traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2m
export TMPDIR=/tmp
b() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 150 python bench.py --gpus 1 "$@" > gpurun_out/r2m/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/r2m/$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/r2m/$n.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("%.3e" % d["value"], "%.3f us/gen" % (d["ms_per_step"]*1e3), c["tile_per_rank"], c["parallelism"], c["schedule"], c["kernel"], "R=%s K=%s" % (c["halo_depth"], c["kernel_depth"]), c["transport"], c["autotune"][:200])')"
}
# config 3 strong-scaled over 8 GPUs: the per-rank strip 4096 x 32768
b s3_local --steps 1000 --warmup 100 --size 4096 --width 32768
b s3_self --steps 1000 --warmup 100 --size 4096 --width 32768 --self-exchange
# config 2 board
b c2 --steps 1000 --warmup 100 --size 8192
# config 4 (65536^2 over 8 GPUs): 2-D 4x2 per-rank tile 32768 x 16384 vs the 1-D strip 8192 x 65536, both through RCCL
b c4_2d_self --steps 640 --warmup 64 --size 32768 --width 16384 --decomp 2d --self-exchange
b c4_1d_self --steps 640 --warmup 64 --size 8192 --width 65536 --self-exchange
b c4_2d_local --steps 640 --warmup 64 --size 32768 --width 16384
# 2x2 vs 1-D P=4 rehearsal (thread ranks sharing the GPU), kernel traces
cd /tmp
R=$GRAFT_REPO_ROOT
for cfg in 2d:2x2:32768 1d:4:32768; do
  tag=$(echo $cfg | tr ':' '_')
  GOL_SCHEDULE=full timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r2m/tr_$tag -o tr -- python $R/tools/rehearse_multirank.py --configs $cfg --gens 640 --warm 64 > $R/gpurun_out/r2m/tr_$tag.log 2>&1 || { echo "trace $cfg failed"; tail -5 $R/gpurun_out/r2m/tr_$tag.log; exit 1; }
  grep '^{' $R/gpurun_out/r2m/tr_$tag.log | cut -c1-200
  python $R/tools/kernel_summary.py $(ls $R/gpurun_out/r2m/tr_$tag/*kernel_trace.csv | head -1) --last-us 20000 | head -14
done

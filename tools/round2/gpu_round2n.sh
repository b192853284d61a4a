#!/bin/bash
# kernel traces of one rank holding the per-rank tiles of configs 3 (strong, 8 GPUs) and 4 (2-D 4x2) with
# halos through a 1-rank RCCL communicator; + the interleaved sub-tile launch order on the driver bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2n
export TMPDIR=/tmp
for i in 1 2 3; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2n/bench_$i.log 2>&1 || exit 1; tail -1 gpurun_out/r2n/bench_$i.log | cut -c170-260; done
cd /tmp
R=$GRAFT_REPO_ROOT
tr() {  # tag, env..., -- bench args
  local tag=$1; shift
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r2n/$tag -o tr -- python $R/bench.py --gpus 1 "$@" > $R/gpurun_out/r2n/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $R/gpurun_out/r2n/$tag.log; exit 1; }
  echo "== $tag: $(tail -1 $R/gpurun_out/r2n/$tag.log | cut -c1-120)"
  python $R/tools/kernel_summary.py $R/gpurun_out/r2n/$tag/tr_kernel_trace.csv --last-us 3000 > $R/gpurun_out/r2n/$tag.summary.txt
  head -12 $R/gpurun_out/r2n/$tag.summary.txt
}
tr bench20 --steps 20 --warmup 5
export GOL_SCHEDULE=split
tr c4_2d_split --steps 320 --warmup 64 --size 32768 --width 16384 --decomp 2d --self-exchange
export GOL_SCHEDULE=full
tr c4_2d_full --steps 320 --warmup 64 --size 32768 --width 16384 --decomp 2d --self-exchange
tr s3_full --steps 640 --warmup 64 --size 4096 --width 32768 --self-exchange
export GOL_SCHEDULE=split
tr s3_split --steps 640 --warmup 64 --size 4096 --width 32768 --self-exchange

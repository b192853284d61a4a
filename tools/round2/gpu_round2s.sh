#!/bin/bash
# full GPU suite; torchrun 2- and 4-process bench sharing the one GPU (host-staged halos: the
# bootstrap/control-plane/collective-autotune path of the driver's multi-GPU run); CLI tile levels A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r2s
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2s/pytest.log 2>&1 || { tail -40 gpurun_out/r2s/pytest.log; exit 1; }
tail -1 gpurun_out/r2s/pytest.log
for P in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $P --master-addr 127.0.0.1 --master-port 2951$P bench.py --gpus $P --steps 64 --warmup 8 --size 8192 --allow-host-staging > gpurun_out/r2s/torchrun_p$P.log 2>&1 || { tail -20 gpurun_out/r2s/torchrun_p$P.log; exit 1; }
  grep '^{' gpurun_out/r2s/torchrun_p$P.log | cut -c1-200; grep -h "RCCL\|host" gpurun_out/r2s/torchrun_p$P.log | head -3
done
for lv in 2 4; do for i in 1 2; do GOL_TILE_LEVELS=$lv timeout -k 10 60 ./build/gol 5 8192 1000 256 0 > gpurun_out/r2s/cfg2_lv$lv_$i.txt || exit 1; echo "lv=$lv $(head -1 gpurun_out/r2s/cfg2_lv$lv_$i.txt)"; done; done

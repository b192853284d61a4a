#!/bin/bash
# The driver's multi-GPU launch line rehearsed on one GPU (ranks share the card: host-staged halos), default board.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2bq
mkdir -p $o
for P in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $P --master-addr 127.0.0.1 --master-port 2961$P bench.py --gpus $P --steps 20 --warmup 5 --allow-host-staging > $o/torchrun_p$P.log 2>&1 || { tail -20 $o/torchrun_p$P.log; exit 1; }
  grep '^{' $o/torchrun_p$P.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("P=%d: %.3e cell-updates/s, %.3f us/gen, n_gpus %d, board %s, %s, R=%s, %s" % ('$P', d["value"], d["ms_per_step"]*1e3, d["n_gpus"], c["board"], c["schedule"], c["halo_depth"], c["transport"]))'
done

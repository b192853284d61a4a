#!/bin/bash
# RCCL p2p channel knobs vs the halo-exchange kernel time (1-rank self-exchange, 32768^2 bench).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/r2aq
mkdir -p $o
run() {  # run <name> <env...>
  local name=$1; shift
  timeout -k 10 200 env "$@" python3 $R/bench.py --gpus 1 --steps 256 --warmup 32 --self-exchange > $o/$name.log 2>&1 || { tail -5 $o/$name.log; return 1; }
  grep '^{"metric"' $o/$name.log | python3 -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("'$name'", "%.3e %.3f us/gen" % (d["value"], d["ms_per_step"]*1e3), c["schedule"], [t for t in c["autotune"].split() if t.startswith("sched")])'
}
prof() {
  local name=$1; shift
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/p_$name -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 128 --warmup 16 --self-exchange > $o/p_$name.log 2>&1 || { tail -5 $o/p_$name.log; return 1; }
  f=$(find $o/p_$name -name '*kernel_stats.csv' | head -1)
  echo "$name $(grep rcclGeneric $f | cut -d, -f3- | cut -c1-80)"
}
run base &&
run minp2p8 NCCL_MIN_P2P_NCHANNELS=8 &&
run perpeer8 NCCL_NCHANNELS_PER_PEER=8 &&
run minp2p8b NCCL_MIN_P2P_NCHANNELS=8 &&
run base2 &&
prof base &&
NCCL_MIN_P2P_NCHANNELS=8 prof minp2p8 &&
NCCL_NCHANNELS_PER_PEER=8 prof perpeer8

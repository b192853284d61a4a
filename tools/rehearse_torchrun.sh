#!/bin/bash
# The driver's multi-GPU launch (torch.distributed.run ... bench.py --gpus 8 --steps 20 --warmup 5) rehearsed with 8 ranks on one GPU (weak, strong, 2d),
# then a 4-rank hang injection with sub-tiles forced on (expected to end non-zero in bounded time)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/rehearse; mkdir -p $O
summ() { python - "$@" <<'PY'
import json,sys
tag=sys.argv[2]
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0])
c=d["config"]
print(tag, "value %.3e"%d["value"], "us/gen", round(d["ms_per_step"]*1e3,2), "board", c["board"], "tile", c["tile_per_rank"], c["parallelism"], "schedule", c["schedule"], "transport", c["transport"], "R", c["halo_depth"])
print("   timing", json.dumps(d.get("timing")))
print("   phases", json.dumps(d.get("phases")))
print("   sched", " ".join(x for x in c["autotune"].split() if x.startswith("sched:")))
PY
}
run8() {
  tag=$1; shift
  start=$(date +%s.%N)
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus 8 --steps 20 --warmup 5 --allow-host-staging "$@" > $O/$tag.json 2> $O/$tag.err
  rc=$?
  end=$(date +%s.%N)
  echo "== $tag: torch.distributed.run --nproc-per-node 8 bench.py --gpus 8 --steps 20 --warmup 5 --allow-host-staging $*" >> $O/summary.txt
  echo "   rc=$rc wall=$(python -c "print(round($end-$start,1))")s" >> $O/summary.txt
  [ $rc -eq 0 ] && summ $O/$tag.json "  " >> $O/summary.txt
  return $rc
}
run8 reh8_weak && run8 reh8_strong --scaling strong && run8 reh8_2d --scaling strong --decomp 2d || { cat $O/summary.txt; exit 1; }
echo "== hang injection: GOL_FAULT=3:10:hang GOL_SUBTILES=2, 4 ranks, --watchdog 10" >> $O/summary.txt
start=$(date +%s.%N)
GOL_FAULT=3:10:hang GOL_SUBTILES=2 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29911 bench.py --gpus 4 --steps 20 --warmup 5 --allow-host-staging --watchdog 10 > $O/hang4.out 2> $O/hang4.err
rc=$?
end=$(date +%s.%N)
echo "   rc=$rc wall=$(python -c "print(round($end-$start,1))")s (expected non-zero, well under the 240 s limit)" >> $O/summary.txt
grep -h "watchdog\|GOL_FAULT\|subtiles\|exitcode\|failed" $O/hang4.err | head -12 | sed 's/^/   /' >> $O/summary.txt
cat $O/summary.txt

#!/bin/bash
# Spread of the driver command with the 12 + 8 cut: pass order 12, 8 (desc) vs 8, 12 (asc), 12 runs each, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2bc
mkdir -p $o
: > $o/all.txt
for i in $(seq 1 12); do
  for ord in desc asc; do
    timeout -k 10 120 env GOL_PASS_ORDER=$ord python bench.py --gpus 1 --steps 20 --warmup 5 > $o/${ord}_$i.log 2>&1 || exit 1
    grep '^{"metric"' $o/${ord}_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("'$ord' %.3f" % (d["ms_per_step"]*1e3))' >> $o/all.txt
  done
done
for ord in desc asc; do echo "$ord: $(grep "^$ord" $o/all.txt | cut -d' ' -f2 | sort -n | tr '\n' ' ')"; done

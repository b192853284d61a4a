#!/bin/bash
# Driver command x8 (spread of the 20-step figure with the 12 + 8 cut).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2ba
mkdir -p $o
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/b20_$i.log 2>&1 || exit 1
  grep '^{"metric"' $o/b20_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); c=d["config"]; print("%.3f us/gen %.3e" % (d["ms_per_step"]*1e3, d["value"]), [t for t in c["autotune"].split() if t.startswith(("pass8","pass12","pass4"))])'
done

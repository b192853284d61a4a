#!/bin/bash
# Driver command x16 (frequency of slow runs with the final build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r2bk
mkdir -p $o
: > $o/all.txt
for i in $(seq 1 16); do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $o/b20_$i.log 2>&1 || exit 1
  grep '^{"metric"' $o/b20_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print("%.3f" % (d["ms_per_step"]*1e3))' >> $o/all.txt
done
sort -n $o/all.txt | tr '\n' ' '; echo

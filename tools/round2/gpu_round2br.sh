#!/bin/bash
# Kernel trace of the driver command with halos through RCCL self-exchange: where the ~30 us of the exchange go.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/r2br
mkdir -p $o
timeout -k 10 200 rocprofv3 --kernel-trace -d $o/p -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --self-exchange > $o/b.log 2>&1 || { tail -5 $o/b.log; exit 1; }
f=$(find $o/p -name '*kernel_trace.csv' | head -1)
cp $f $o/kernel_trace.csv
python3 - $o/kernel_trace.csv <<'PY'
import csv, sys
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]) for r in csv.DictReader(open(sys.argv[1])))
end = max(e for _, e, _, _ in rows)
t0 = end - 700e3
for s, e, q, k in rows:
    if s >= t0:
        n = k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].replace("gol::hipk::", "")
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{q} {n[:60]}")
PY
grep '^{"metric"' $o/b.log | cut -c1-150

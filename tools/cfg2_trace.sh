#!/bin/bash
# Kernel trace of the BASELINE config-2 CLI run (gol 5 8192 1000 256 0): GPU idle between step
# kernels (graph replays vs eager launches).  Output: gpurun_out/cfg2_trace/*.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/cfg2_trace
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/cfg2_trace -o cli -- $R/build/gol 5 8192 1000 256 0 > $R/gpurun_out/cfg2_trace/cli.log 2>&1 || exit 3
f=$(find $R/gpurun_out/cfg2_trace -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_gaps.py $f 60 > $R/gpurun_out/cfg2_trace/gaps.txt
cat $R/gpurun_out/cfg2_trace/cli.log $R/gpurun_out/cfg2_trace/gaps.txt
python3 - "$f" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
st = [r for r in rows if "step_" in r["Kernel_Name"]][-60:]
prev = None
for r in st:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = (s - prev) / 1e3 if prev else 0
    print(f"{(e - s) / 1e3:8.1f} us  gap {g:7.1f} us  {r['Kernel_Name'][:60]}")
    prev = e
PY

#!/usr/bin/env python3
"""Per-kernel durations and overlap from a rocprofv3 kernel_trace.csv (last N dispatches)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "step_" in r["Kernel_Name"]][-n:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    name = r["Kernel_Name"].split("(")[0].split("::")[-1][:40]
    print(f"{name:42s} grid={r['Grid_Size_X']:>8s} q={r.get('Queue_Id','?'):>3s} start={s/1e3:9.1f}us end={e/1e3:9.1f}us dur={(e-s)/1e3:7.1f}us")

#!/usr/bin/env python3
"""Last N dispatches of a rocprofv3 kernel_trace.csv with start/end/duration and the gap to the
previous dispatch end (us): python tools/trace_tail.py <kernel_trace.csv> [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("gol::hipk::", "")[:48]
    print(f"{name:48s} q={r['Queue_Id']:>2s} grid={r['Grid_Size_X']:>8s} s={s/1e3:9.1f} e={e/1e3:9.1f} "
          f"d={(e-s)/1e3:7.1f} gap={gap:7.1f}")
    prev = e if prev is None else max(prev, e)

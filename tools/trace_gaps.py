#!/usr/bin/env python3
"""GPU idle between consecutive kernels of a rocprofv3 kernel_trace.csv: gap histogram, the
gaps, and busy/span over the step kernels of the run (eager launches vs graph replays)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
step = [k for k in ks if "step_" in k[2]]
if len(sys.argv) > 2:  # only the last N step kernels (e.g. the timed region of a bench run)
    step = step[-int(sys.argv[2]):]
gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(step, step[1:])]
busy = sum(e - s for s, e, _ in step) / 1e3
span = (step[-1][1] - step[0][0]) / 1e3
print(f"{len(step)} step-kernel dispatches, busy {busy:.1f} us of span {span:.1f} us ({busy / span:.4f})")
for lo, hi in [(0, 1), (1, 5), (5, 10), (10, 20), (20, 50), (50, 1e9)]:
    sel = [g for g in gaps if lo <= g < hi]
    print(f"  gaps {lo:>4}-{hi:<6g} us: {len(sel):4d}  total {sum(sel):9.1f} us")
durs = [(e - s) / 1e3 for s, e, _ in step]
n = len(durs)
for name, part in [("first 10%", durs[: n // 10]), ("last 50%", durs[n // 2:])]:
    if part:
        print(f"  kernel duration {name}: mean {sum(part) / len(part):.1f} us")

#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 kernel_trace.csv: dispatches, total / mean duration per kernel
name, and the GPU's busy time (union of kernel intervals) over the traced span.

    python tools/kernel_summary.py <kernel_trace.csv> [--after-us T]   (skip the first T us: init)
"""
import argparse
import csv
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--after-us", type=float, default=0.0)
ap.add_argument("--last-us", type=float, default=0.0, help="only the last T us of the trace (the timed region)")
a = ap.parse_args()
rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(a.trace))]
rows.sort()
t0 = rows[0][0] + a.after_us * 1e3
if a.last_us > 0:
    t0 = max(t0, max(e for _, e, _ in rows) - a.last_us * 1e3)
rows = [r for r in rows if r[0] >= t0]
agg = defaultdict(lambda: [0, 0.0])
for s, e, k in rows:
    name = k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].replace("gol::hipk::", "")
    agg[name][0] += 1
    agg[name][1] += (e - s) / 1e3
busy, cur_s, cur_e = 0.0, None, None
for s, e, _ in rows:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += (cur_e - cur_s) / 1e3
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
if cur_e is not None:
    busy += (cur_e - cur_s) / 1e3
span = (max(e for _, e, _ in rows) - rows[0][0]) / 1e3 if rows else 0.0
print(f"{len(rows)} dispatches; GPU busy (union) {busy:.1f} us of span {span:.1f} us ({busy / max(span, 1e-9):.3f})")
print(f"{'kernel':70s} {'n':>6s} {'total us':>11s} {'mean us':>9s}")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{k[:70]:70s} {n:6d} {t:11.1f} {t / n:9.2f}")

#!/usr/bin/env python3
"""Per-queue view of the last T us of a rocprofv3 kernel_trace.csv (the timed region of a run):
for every HIP queue, its step kernels in order with the gap before each, and where the gaps sit
(before a superstep's first, seam-reading pass, ROWS=2, or between passes of a superstep).

    python tools/trace_queues.py <kernel_trace.csv> --last-us T
"""
import argparse
import csv
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--last-us", type=float, required=True)
ap.add_argument("--show", type=int, default=24, help="kernels listed per queue")
a = ap.parse_args()
rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]) for r in csv.DictReader(open(a.trace))]
end = max(e for _, e, _, _ in rows)
t0 = end - a.last_us * 1e3
rows = sorted(r for r in rows if r[0] >= t0 and "step_" in r[3])
byq = defaultdict(list)
for r in rows:
    byq[r[2]].append(r)
for q, ks in byq.items():
    gaps_seam, gaps_mid = [], []
    print(f"== queue {q}: {len(ks)} step kernels")
    for i, (s, e, _, k) in enumerate(ks):
        name = k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].replace("gol::hipk::", "")
        gap = (s - ks[i - 1][1]) / 1e3 if i else 0.0
        if i:
            (gaps_seam if ", 2>" in name else gaps_mid).append(gap)
        if i < a.show:
            print(f"  {(s - t0) / 1e3:9.1f} {gap:7.1f} {(e - s) / 1e3:7.1f}  {name}")
    busy = sum(e - s for s, e, _, _ in ks) / 1e3
    span = (ks[-1][1] - ks[0][0]) / 1e3
    print(f"  busy {busy:.1f} of span {span:.1f} us; gaps before seam passes: n={len(gaps_seam)} total {sum(gaps_seam):.1f} us "
          f"(mean {sum(gaps_seam) / max(1, len(gaps_seam)):.1f}); other gaps: n={len(gaps_mid)} total {sum(gaps_mid):.1f} us")

#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel (averages per dispatch)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
agg = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for r in rows:
    k = r["Kernel_Name"]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
for k, v in agg.items():
    d = len(disp[k])
    v = {c: x / d for c, x in v.items()}
    print(f"{k[:90]}  dispatches={d}")
    for c, x in sorted(v.items()):
        print(f"    {c:24s} {x:14.4g}")
    if "GRBM_GUI_ACTIVE" in v and "SQ_INSTS_VALU" in v:
        cyc = v["GRBM_GUI_ACTIVE"] / 8
        print(f"    kernel cycles per XCD  {cyc:.4g}; VALU issue utilisation {v['SQ_INSTS_VALU'] * 2 / (cyc * 1024):.3f}")
    if "SQ_WAVE_CYCLES" in v and "SQ_ACTIVE_INST_ANY" in v:
        w = v["SQ_WAVE_CYCLES"]
        print(f"    wave time: active {v['SQ_ACTIVE_INST_ANY']/w:.3f}  wait(waitcnt) {v.get('SQ_WAIT_ANY',0)/w:.3f}"
              f"  wait(inst) {v.get('SQ_WAIT_INST_ANY',0)/w:.3f}")

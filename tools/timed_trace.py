#!/usr/bin/env python3
"""Timeline of a bench's timed run from a rocprofv3 trace (``--kernel-trace --marker-trace``, bench run
with GOL_ROCTX=1 and --no-phases): the LAST ``gol.run`` roctx range is the timed run.  Prints every
kernel from the range start until the first kernel of the population readout, per queue, with its
start offset from the range start, duration and the gap before it, then a summary: host-to-first-
kernel latency, GPU busy (union of intervals) and idle inside the run, and the end of the last kernel.

    python tools/timed_trace.py <rocprofv3 output dir>
"""
import csv
import glob
import os
import sys


def rows(pattern_dir, suffix):
    fs = glob.glob(os.path.join(pattern_dir, "**", f"*{suffix}"), recursive=True)
    if not fs:
        sys.exit(f"no *{suffix} under {pattern_dir}")
    out = []
    for f in fs:
        out += list(csv.DictReader(open(f)))
    return out


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("gol::hipk::", "")
    return n.split("(")[0][:60]


def main():
    d = sys.argv[1]
    ks = rows(d, "kernel_trace.csv")
    ms = rows(d, "marker_api_trace.csv")
    runs = [m for m in ms if any("gol.run" == str(v) for v in m.values())]
    if not runs:
        sys.exit("no gol.run roctx range (run the bench with GOL_ROCTX=1 under --marker-trace)")
    r = max(runs, key=lambda m: int(m["Start_Timestamp"]))
    t0, t_host_end = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    kern = sorted((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Queue_Id"], short(k["Kernel_Name"])) for k in ks)
    sel = []
    for s, e, q, n in kern:
        if s < t0:
            continue
        if "reduce" in n or "copyBuffer" in n or "fillBuffer" in n:
            break
        sel.append((s, e, q, n))
    if not sel:
        sys.exit("no kernels after the range start")
    print(f"timed run: host range {(t_host_end - t0) / 1e3:.1f} us (run() call), {len(sel)} kernels")
    last = {}
    for s, e, q, n in sel:
        gap = (s - last[q]) / 1e3 if q in last else (s - t0) / 1e3
        last[q] = e
        print(f"  q{q:>3} {(s - t0) / 1e3:8.1f} +{(e - s) / 1e3:7.1f}  gap {gap:6.1f}  {n}")
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in sorted(sel):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    first, end = sel[0][0], max(e for _, e, _, _ in sel)
    print(f"first kernel starts {(first - t0) / 1e3:.1f} us after run() was entered; last kernel ends at {(end - t0) / 1e3:.1f} us")
    # host side of the first launch (sub-tile supersteps mark it): run() entry -> launch call -> its return
    for tag in ("gol.launch0", "gol.launch0_done"):
        mk = [m for m in ms if any(tag == str(v) for v in m.values()) and t0 <= int(m["Start_Timestamp"]) <= t_host_end]
        if mk:
            print(f"  {tag}: {(int(mk[0]['Start_Timestamp']) - t0) / 1e3:.1f} us after run() was entered")
    print(f"GPU busy {busy / 1e3:.1f} us of the {(end - first) / 1e3:.1f} us from first start to last end "
          f"(idle {(end - first - busy) / 1e3:.1f} us)")


if __name__ == "__main__":
    main()

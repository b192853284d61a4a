#!/usr/bin/env python3
"""One summary line of a bench.py JSON record (stdin): us/generation, rate, schedule, kernel, the
init-time prediction when present, and the schedule timings of the autotune string.

    python3 bench.py ... | python3 tools/bench_line.py "<label>"
"""
import json
import sys


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else ""
    d = json.loads(sys.stdin.read().strip().splitlines()[-1])
    if d.get("value") is None:
        print(f"[{label}] error: {d.get('error')}")
        return
    c = d["config"]
    sched = " ".join(t for t in c.get("autotune", "").split() if t.startswith("sched:"))
    pred = d.get("sched_predicted_us_per_gen")
    print(f"[{label}] {d['ms_per_step'] * 1e3:.3f} us/gen {d['value']:.3e} {c['schedule']} {c['kernel']} "
          f"R {c['halo_depth']} graphs {c['graph_launches']}"
          + (f" predicted {pred:.3f}" if pred else "") + (f" {sched}" if sched else ""))


if __name__ == "__main__":
    main()

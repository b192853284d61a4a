#!/usr/bin/env python3
"""Short-run overhead probe (the driver's bench: 20 timed generations after 5 warmup ones).

For each engine variant, times `reps` back-to-back timed regions exactly as bench.py does
(device sync + t0, step(n), device sync, t1) and prints median / min us per generation, plus the
split between host enqueue time (step() return) and the wait for the GPU."""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=32768)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--variants", default="sub2,sub0,sub2-nograph,sub0-nograph")
    ap.add_argument("--torch-sync", action="store_true")
    args = ap.parse_args()
    import gol_amd

    if args.torch_sync:
        import torch
    for v in args.variants.split(","):
        kw = {}
        if v.startswith("sub2"):
            kw["subtiles"] = 2
        elif v.startswith("sub0"):
            kw["subtiles"] = 0
        if "nograph" in v:
            kw["graph"] = False
        if "r32" in v:
            kw["halo_depth"] = 32
        sim = gol_amd.Simulation(args.size, backend="hip", device=0, run_hint=args.steps, **kw).init(5, seed=1)
        sim.step(5)
        sim.synchronize()
        walls, enq = [], []
        for _ in range(args.reps):
            sim.synchronize()
            if args.torch_sync:
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            sim.step(args.steps)
            t1 = time.perf_counter()
            sim.synchronize()
            if args.torch_sync:
                torch.cuda.synchronize()
            t2 = time.perf_counter()
            walls.append((t2 - t0) / args.steps * 1e6)
            enq.append((t1 - t0) * 1e6)
        st = sim.stats()
        print(json.dumps({"variant": v, "schedule": st["schedule"], "graph_launches": st["graph_launches"],
                          "median_us_per_gen": round(statistics.median(walls), 3), "min_us_per_gen": round(min(walls), 3),
                          "median_enqueue_us": round(statistics.median(enq), 1), "tuning": st["tuning"]}), flush=True)
        del sim


if __name__ == "__main__":
    main()

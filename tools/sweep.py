#!/usr/bin/env python3
"""In-process parameter sweep of the single-GPU engine (interleaved rounds, one process, so the
variants see the same device and clocks — cdna_hip_programming.md §5.4 rule 24).

    python tools/sweep.py --size 32768 --gens 800 --depth 4,6,8,12 --waves 0,4096 --rounds 2
Prints one line per (variant, round) and a median summary as JSON lines.
"""
import argparse
import itertools
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ints(s):
    return [int(x) for x in s.split(",") if x != ""]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=32768)
    ap.add_argument("--gens", type=int, default=800)
    ap.add_argument("--depth", type=ints, default=[8])
    ap.add_argument("--waves", type=ints, default=[0])
    ap.add_argument("--rows", type=ints, default=[0])
    ap.add_argument("--kernel", default="temporal")
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()

    import gol_amd

    variants = list(itertools.product(args.depth, args.waves, args.rows))
    results = {v: [] for v in variants}
    for rnd in range(args.rounds):
        for v in variants:
            depth, waves, rows = v
            sim = gol_amd.Simulation(args.size, backend="hip", device=0, halo_depth=depth, waves_target=waves,
                                     rows_per_wave=rows, kernel=args.kernel).init(5, seed=7)
            sim.step(max(depth * 40, 64))
            sim.synchronize()
            t0 = time.perf_counter()
            sim.step(args.gens)
            sim.synchronize()
            dt = time.perf_counter() - t0
            st = sim.stats()
            rate = args.size * args.size * args.gens / dt
            results[v].append(rate)
            print(json.dumps({"round": rnd, "depth": depth, "waves_target": waves, "rows": rows,
                              "plan_waves": st["plan_waves"], "lane_eff": round(st["lane_efficiency"], 4),
                              "us_per_gen": dt / args.gens * 1e6, "cells_per_s": rate}), flush=True)
            del sim
    for v, rs in results.items():
        print(json.dumps({"summary": True, "depth": v[0], "waves_target": v[1], "rows": v[2],
                          "median_cells_per_s": statistics.median(rs), "max": max(rs)}), flush=True)


if __name__ == "__main__":
    main()

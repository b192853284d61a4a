#!/usr/bin/env python3
"""Multi-rank engine overhead on ONE GPU: P thread ranks with the RCCL-semantics device transport
(GOL_TRANSPORT=p2p: device halo buffers, stream-ordered copies, per-peer FIFO matching) share the
card, so their aggregate throughput against one rank on the same global board measures what the
multi-rank superstep costs (extra ghost-row compute, halo packing and copies, cross-stream events,
P engines' launches) apart from the xGMI link itself.

    python tools/rehearse_multirank.py [--gens 1280] [--configs 1d:2:32768,2d:2x2:32768,...]
Prints one JSON line per configuration.
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(gol, decomp, grid, P, N, gens, warm):
    ts = gol.parallel.p2p_thread_transports(P) if P > 1 else [gol.native.SelfTransport()]
    bar = threading.Barrier(P)
    res, errs, sims = [None] * P, [], [None] * P

    def rank_main(r):
        try:
            s = gol.Simulation(N, ts[r], backend="hip", device=0, global_mode=True, decomp=decomp, grid=grid)
            s.init(5, seed=7)
            sims[r] = s
            s.step(warm)
            s.synchronize()
            bar.wait()
            t0 = time.perf_counter()
            s.step(gens)
            s.synchronize()
            bar.wait()
            res[r] = (time.perf_counter() - t0, s.stats(), s.fingerprint())
        except Exception as e:  # reported below
            errs.append(repr(e))
            bar.abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    if errs:
        raise RuntimeError(errs)
    el = max(x[0] for x in res)
    st = res[0][1]
    return {
        "decomp": decomp if P > 1 else "single",
        "grid": grid,
        "P": P,
        "board": N,
        "gens": gens,
        "us_per_gen": el / gens * 1e6,
        "cell_updates_per_s": N * N * gens / el,
        "rank0": {k: st[k] for k in ("depth", "kernel_depth", "kernel", "schedule") if k in st},
        "fingerprints": sorted({x[2] for x in res}),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gens", type=int, default=1280)
    ap.add_argument("--warm", type=int, default=128)
    ap.add_argument("--configs", default="single:1:32768,1d:2:32768,2d:2x2:32768,1d:4:32768,single:1:65536,2d:4x2:65536")
    args = ap.parse_args()
    import gol_amd as gol

    for spec in args.configs.split(","):
        kind, p, n = spec.split(":")
        if kind == "single":
            P, decomp, grid = 1, "1d", ""
        elif kind == "1d":
            P, decomp, grid = int(p), "1d", ""
        else:
            px, py = (int(v) for v in p.split("x"))
            P, decomp, grid = px * py, "2d", p
        out = run(gol, decomp, grid, P, int(n), args.gens, args.warm)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

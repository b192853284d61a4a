#!/usr/bin/env python3
"""Where the init-time prediction and bench.py's measurement differ (one GPU).

Builds the bench's simulation (same arguments as bench.py's single-rank path), then times the hinted run
several ways, each bracketed as bench.py brackets its timed run (engine device barrier, perf_counter, the
run, torch.cuda.synchronize()):

  bench      after a `--warmup` run, as bench.py does
  again      right after the previous timed run (no warmup run in between)
  cxx        the same bracket timed in C++ (Engine::time_runs: what the init-time prediction runs)
  idle<ms>   after sleeping that long with the GPU idle (clock state)
  noop       an empty run (sim.step(0)): the Python + pybind + sync floor

    python tools/predict_gap.py [--size 32768] [--width 0] [--steps 20] [--warmup 5] [--self-exchange]
"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=32768)
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--self-exchange", action="store_true")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch

    import gol_amd

    native = gol_amd.native
    if a.self_exchange:
        native.hip_set_device(0)
        transport = native.make_rccl_transport(native.SelfTransport())
    else:
        transport = native.SelfTransport()
    torch.cuda.synchronize()
    sim = gol_amd.Simulation(a.size, transport, backend="hip", device=0, run_hint=a.steps,
                             self_exchange=a.self_exchange, width=a.width, watchdog=120.0)
    sim.init(pattern=5, seed=0x5EED)
    st = sim.stats()
    print(f"schedule {st['schedule']} kernel {st['kernel']} predicted {st['predicted_us_per_gen']:.3f} us/gen "
          f"over {st['predicted_gens']} gens", flush=True)

    def timed(gens):
        sim.synchronize()
        torch.cuda.synchronize()
        sim.engine.device_barrier()
        t0 = time.perf_counter()
        sim.step(gens)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6

    res = {k: [] for k in ("bench", "again", "cxx", "idle1", "idle10", "idle100", "noop")}
    for _ in range(a.reps):
        sim.step(a.warmup)
        res["bench"].append(timed(a.steps) / a.steps)
        res["again"].append(timed(a.steps) / a.steps)
        res["cxx"].extend(sim.engine.time_runs(a.steps, 1))  # the same bracket in C++ (the prediction's)
        for ms in (1, 10, 100):
            sim.synchronize()
            time.sleep(ms / 1e3)
            t0 = time.perf_counter()
            sim.step(a.steps)
            torch.cuda.synchronize()
            res[f"idle{ms}"].append((time.perf_counter() - t0) * 1e6 / a.steps)
        res["noop"].append(timed(0))
    for k, v in res.items():
        unit = "us per run" if k == "noop" else "us/gen"
        print(f"  {k:8s} median {statistics.median(v):8.3f} {unit}  ({', '.join(f'{x:.3f}' for x in v)})", flush=True)
    sim.synchronize()
    del sim, transport


if __name__ == "__main__":
    main()

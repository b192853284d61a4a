#!/usr/bin/env python3
"""Headline benchmark: cell-updates/sec (whole node) on a 32768^2 board per GPU.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A *step* is one Game of Life generation (B3/S23) over the whole board.  Each rank owns one GPU and a
32768 x 32768 tile (weak scaling, the reference's per-rank semantics: gol-main.c:76) — the global
board is (N*32768) x 32768, a torus, with RCCL halo exchange over xGMI between ranks.  ``--scaling
strong`` instead splits one 32768^2 board over the N GPUs.  The board is random (pattern 5,
synthetic).  The timed region runs every generation in full: W untimed warmup generations, then the
ranks are aligned (host barrier + a 1-element RCCL all-reduce on the engine's stream, waited for on
every GPU), K timed generations, device sync; the max over ranks of the per-rank elapsed time is
reported, with the residual start skew (``start_skew_us``).  Metric = global cells x K / elapsed.
``--gpus N`` without a launcher (no WORLD_SIZE) starts ``torch.distributed.run`` with N ranks as a
child process and relays its output (it never measures one GPU in place of N).  A progress watchdog
(``--watchdog`` seconds) makes every rank exit non-zero if a peer hangs or RCCL fails.  Without a
GPU it falls back to the CPU backend on BASELINE config 1 (256^2).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "cell-updates/sec (whole node) on 32768^2 board; 1/2/4/8-GPU weak+strong scaling"


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4000, help="timed generations")
    ap.add_argument("--warmup", type=int, default=400, help="untimed generations")
    ap.add_argument("--size", type=int, default=32768, help="tile side per GPU (weak) / board side (strong)")
    ap.add_argument("--width", type=int, default=0,
                    help="board columns (0 = --size: square); e.g. one GPU holding another config's per-rank tile")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    ap.add_argument("--decomp", default="1d", help="1d | 2d | auto")
    ap.add_argument("--halo-depth", type=int, default=int(os.environ.get("GOL_HALO_DEPTH", "0")),
                    help="generations per halo exchange (0 = auto: 32 without neighbours; 128 for 1-D strips "
                         "of >= 2048 rows with neighbours and for sub-tile ranks; 56 for 2-D tiles of >= 2048 rows)")
    ap.add_argument("--kernel-depth", type=int, default=int(os.environ.get("GOL_KERNEL_DEPTH", "0")),
                    help="generations per kernel pass (0 = auto)")
    ap.add_argument("--kernel", default=os.environ.get("GOL_KERNEL", "auto"),
                    help="auto (timed at init) | temporal | tile | lds")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--yardstick", action="store_true", help="also time the naive byte-per-cell kernel (rank 0)")
    ap.add_argument("--self-exchange", action="store_true",
                    help="route the halos of directions whose neighbour is the rank itself through the transport "
                         "(one GPU: a 1-rank RCCL communicator, ncclSend/ncclRecv to itself)")
    ap.add_argument("--allow-host-staging", action="store_true",
                    help="if RCCL cannot initialise (e.g. ranks sharing one GPU in a rehearsal), stage halos "
                         "through host memory instead of failing")
    ap.add_argument("--watchdog", type=float, default=float(os.environ.get("GOL_WATCHDOG", "120")),
                    help="seconds without progress (or an RCCL error) before every rank aborts non-zero (0 = off)")
    ap.add_argument("--no-phases", action="store_true", help="skip the untimed per-phase probe after the run")
    ap.add_argument("--seed", type=int, default=0x5EED)
    return ap.parse_args(argv)


def rank_problems(ranks, P, rccl_ranks):
    """Why a multi-rank record is not a valid measurement: the ranks ran different schedules or halo
    depths (their exchanges would not match), or the RCCL communicator does not span every rank
    (rccl_ranks None: no RCCL data plane).  The kernel is tuned per rank on its own GPU and may differ
    (per_rank_kernel reports it): 8 processes timing kernels at once on one GPU picked four different
    ones in the rehearsal, a difference of timing noise, not of the measurement's validity."""
    problems = []
    if len({(r["schedule"], r["depth"]) for r in ranks}) > 1:
        problems.append("ranks disagree on the schedule: " +
                        ", ".join(f"{i}:{r['schedule']}/{r['kernel']}/{r['depth']}" for i, r in enumerate(ranks)))
    if rccl_ranks is not None and P > 1 and rccl_ranks != P:
        problems.append(f"the RCCL communicator spans {rccl_ranks} of {P} ranks")
    return problems


def prediction_fields(predicted_us, measured_us):
    """The engine's init-time prediction of this run next to the measurement: the chosen schedule timed at
    the end of init the way the run executes it (same supersteps, graph replay or eager launches, after a
    device barrier, from an idle GPU; median of a few samples, max over ranks).  None where the backend
    does not measure one (CPU)."""
    p = round(float(predicted_us), 3) if predicted_us else None
    return {"sched_predicted_us_per_gen": p,
            "predicted_over_measured": round(p / measured_us, 4) if p and measured_us > 0 else None}


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_children(args) -> int:
    """``--gpus N`` (N > 1) without a launcher: run this script under torch.distributed.run, N ranks,
    as a child process (never exec: the parent touches no GPU, but a child keeps the contract simple),
    and relay its exit code.  The ranks print the JSON line themselves (rank 0)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] --gpus {args.gpus} without a launcher: running {' '.join(cmd[1:6])} ... as a child",
          file=sys.stderr, flush=True)
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


_RECORD = None


def _reserve_stdout():
    """Keep a private handle on stdout for the JSON record and point file descriptor 1 at stderr."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(fd, "w", buffering=1)


def emit(record) -> None:
    """Print the one JSON line (to the real stdout)."""
    out = _RECORD if _RECORD is not None else sys.stdout
    out.write(json.dumps(record) + "\n")
    out.flush()


def main() -> int:
    args = parse_args()
    # Decided before anything touches the GPU (importing the package does not; hip_device_count does).
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        return launch_children(args)
    world = int(world_env or "1")
    if world != args.gpus:
        msg = f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks"
        print(f"[bench] error: {msg}", file=sys.stderr, flush=True)
        if os.environ.get("RANK", "0") == "0":  # the one-JSON-line contract holds for failures too
            print(json.dumps({"metric": METRIC, "value": None, "unit": "cell-updates/s", "n_gpus": world,
                              "error": msg}), flush=True)
        return 2

    # stdout carries the JSON record only: what C libraries write to it (RCCL prints a version block at
    # communicator init) goes to stderr from here on
    global _RECORD
    _RECORD = _reserve_stdout()

    import gol_amd
    from gol_amd.parallel import init_distributed, rccl_transport, torch_transport

    native = gol_amd.native
    have_gpu = native.hip_device_count() > 0
    backend = "hip" if have_gpu else "cpu"
    size, steps, warmup = args.size, args.steps, args.warmup
    if not have_gpu:
        size, steps, warmup = 256, min(steps, 100), min(warmup, 10)

    rank, P, local, cpu_group = init_distributed()
    rccl = None
    if P > 1:
        control = torch_transport(cpu_group)
        transport = control
        if backend == "hip":
            import torch
            import torch.distributed as dist

            try:
                rccl = rccl_transport(control, group=cpu_group)
            except Exception as e:
                print(f"[bench] rank {rank}: RCCL transport unavailable ({e})", file=sys.stderr, flush=True)
            ok = torch.tensor([1 if rccl is not None else 0], dtype=torch.int32)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=cpu_group)  # every rank must agree
            if int(ok.item()) == 1:
                transport = rccl
            elif not args.allow_host_staging:
                # a multi-GPU number measured over host-staged halos is not the RCCL/xGMI design
                if rank == 0:
                    emit({"metric": METRIC, "value": None, "unit": "cell-updates/s", "n_gpus": P,
                          "error": "RCCL unavailable on some rank; refusing to measure host-staged "
                                   "halos (pass --allow-host-staging to do so)"})
                return 3
            elif rank == 0:
                print("[bench] using host-staged halos on every rank", file=sys.stderr, flush=True)
    elif args.self_exchange and backend == "hip":
        native.hip_set_device(0)
        rccl = native.make_rccl_transport(native.SelfTransport())
        transport = rccl
    else:
        transport = native.SelfTransport()

    import torch

    use_torch_sync = backend == "hip" and torch.cuda.is_available()
    if use_torch_sync:
        # torch's lazy device initialisation (its first synchronize) before the engine's init: the
        # engine's init ends by spinning the GPU up to its steady clock (GOL_SPINUP_MS), and the
        # warmup and timed run should follow it without an idle gap
        torch.cuda.synchronize()

    t_init = time.perf_counter()
    sim = gol_amd.Simulation(
        size,
        transport,
        backend=backend,
        global_mode=(args.scaling == "strong"),
        decomp=args.decomp,
        halo_depth=args.halo_depth,
        kernel_depth=args.kernel_depth,
        graph=not args.no_graph,
        overlap=not args.no_overlap,
        kernel=args.kernel,
        device=local if backend == "hip" else None,
        run_hint=steps,  # the timed run replays one captured graph (graph boundaries idle the GPU)
        self_exchange=args.self_exchange,
        width=args.width if have_gpu else 0,
        watchdog=args.watchdog,
    )
    sim.init(pattern=5, seed=args.seed)
    my_init = time.perf_counter() - t_init
    init_s = transport.allreduce_max(my_init)
    init_per_rank = [round(my_init, 3)]
    if P > 1:
        import torch.distributed as dist

        init_per_rank = [None] * P
        dist.all_gather_object(init_per_rank, round(my_init, 3), group=cpu_group)
    dec = sim.decomposition
    cells = dec.H * dec.W

    # The timed run ends with torch.cuda.synchronize() alone: hipDeviceSynchronize waits for every stream
    # of the device, the engine's two included (tools/sync_check.py checks it), and a hang is still
    # caught (the watchdog fires on GPU work outstanding without progress).  The engine's own stream
    # syncs before it cost ~6.6 us per run: driver command 11.29 vs 11.62 us/gen, mean of 10 alternating
    # pairs (profiles/end_sync_round3.txt).  BENCH_END_SYNC=both restores them (measurement knob).
    end_sync = os.environ.get("BENCH_END_SYNC", "torch")

    def device_sync(end=False):
        if not (end and use_torch_sync and end_sync == "torch"):
            sim.synchronize()  # the engine's own HIP streams (watchdog-armed)
        if use_torch_sync:
            torch.cuda.synchronize()

    device_sync()
    sim.step(warmup)
    device_sync()
    sim.engine.device_barrier()  # host barrier + RCCL all-reduce completed on every GPU
    t0 = time.perf_counter()
    sim.step(steps)
    device_sync(end=True)
    t1 = time.perf_counter()
    elapsed = transport.allreduce_max(t1 - t0)
    # perf_counter is CLOCK_MONOTONIC: comparable across the processes of one node
    start_skew = transport.allreduce_max(t0) - transport.allreduce_min(t0)
    span = transport.allreduce_max(t1) - transport.allreduce_min(t0)
    transport.barrier()

    def gather(obj):
        """Every rank's value, in rank order (rank 0 reports them)."""
        if P == 1:
            return [obj]
        import torch.distributed as dist

        out = [None] * P
        dist.all_gather_object(out, obj, group=cpu_group)
        return out

    t0_min = transport.allreduce_min(t0)
    per_rank = gather({"elapsed_us": round((t1 - t0) * 1e6, 2), "t0_offset_us": round((t0 - t0_min) * 1e6, 2)})
    pop = sim.population()
    st = sim.stats()
    halo_bytes = transport.allreduce_sum(int(st["halo_bytes"]))  # all ranks, init + warmup + timed
    k_timed = st["depth"] if steps >= st["depth"] else steps
    phases = None
    if backend == "hip" and not args.no_phases:
        ph = sim.engine.phase_probe(min(steps, st["depth"]))
        phases = {"superstep_gens": int(ph.get("superstep_gens", k_timed)),
                  "timed_supersteps": -(-steps // max(1, int(ph.get("superstep_gens", k_timed))))}
        for key in ("exchange_us", "superstep_us"):
            if key in ph:
                phases[key + "_max"] = round(transport.allreduce_max(ph[key]), 2)
                phases[key + "_min"] = round(transport.allreduce_min(ph[key]), 2)

    # Per-rank diagnosis of the first multi-GPU records: every rank's timing, probe
    # phases and chosen schedule; a run whose ranks disagree on the schedule, or whose RCCL
    # communicator does not span every rank, is an error record (non-zero exit), not a number.
    mine = {"schedule": st["schedule"], "kernel": st["kernel"], "depth": st["depth"],
            "kernel_depth": st["kernel_depth"],
            "exchange_us": round(ph["exchange_us"], 2) if phases is not None and "exchange_us" in ph else None,
            "superstep_us": round(ph["superstep_us"], 2) if phases is not None and "superstep_us" in ph else None}
    ranks = gather(mine)
    problems = rank_problems(ranks, P, transport.data_plane_ranks() if rccl is not None else None)
    per_rank_block = {
        "per_rank_elapsed_us": [r["elapsed_us"] for r in per_rank],
        "per_rank_t0_offset_us": [r["t0_offset_us"] for r in per_rank],
        "per_rank_exchange_us": [r["exchange_us"] for r in ranks],
        "per_rank_superstep_us": [r["superstep_us"] for r in ranks],
        "per_rank_schedule": [r["schedule"] for r in ranks],
        "per_rank_kernel": [r["kernel"] for r in ranks],
        "per_rank_depth": [r["depth"] for r in ranks],
    }
    if problems:
        if rank == 0:
            emit({"metric": METRIC, "value": None, "unit": "cell-updates/s", "n_gpus": P,
                  "error": "; ".join(problems), "per_rank": per_rank_block})
        return 5

    yard = None
    if args.yardstick and rank == 0 and have_gpu:
        ys = min(size, 16384)
        yg = 50
        t, _ = native.naive_byte_run(ys, yg, 256, True, args.seed)
        yard = {"board": ys, "generations": yg, "cell_updates_per_s": ys * ys * yg / t}

    if rank == 0:
        value = cells * steps / elapsed
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "cell-updates/s",
            "n_gpus": P if have_gpu else 0,
            "steps": steps,
            "warmup": warmup,
            "ms_per_step": elapsed / steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u1 bit-packed (64 cells per u64)",
            "data": "synthetic (pattern 5: seeded random board, density 1/2)",
            "config": {
                "model": "Conway B3/S23 torus, bit-packed temporal-blocked HIP kernel",
                "board": [dec.H, dec.W],
                "tile_per_rank": [sim.geometry.h, sim.geometry.w],
                "global_batch": cells,
                "seq_len": None,
                "parallelism": f"{'2d' if dec.Px > 1 else '1d'}-spatial p{P} ({dec.Px}x{dec.Py})",
                "backend": backend,
                "halo_depth": st["depth"],
                "kernel_depth": st["kernel_depth"],
                "kernel": st["kernel"],
                "tile_waves": st["tile_waves"],
                "schedule": st["schedule"],
                "autotune": st["tuning"],
                "graph_launches": st["graph_launches"],
                "plan_waves": st["plan_waves"],
                "lane_efficiency": round(st["lane_efficiency"], 4),
                "population": pop,
                "transport": transport.name(),
                "rccl_nranks": transport.data_plane_ranks() if rccl is not None else None,
                "self_exchange": bool(args.self_exchange),
                "rccl_registered": bool(st.get("registered", False)),
                "halo_exchanges_rank0": st["exchanges"],
                "halo_bytes_all_ranks": halo_bytes,
                "watchdog_s": args.watchdog,
            },
            "timing": {
                "per_rank_elapsed_max_us": round(elapsed * 1e6, 2),
                "start_skew_us": round(start_skew * 1e6, 2),
                "span_us": round(span * 1e6, 2),
                "init_s": round(init_s, 3),
                "init_s_per_rank": init_per_rank,
            },
            "start_skew_us": round(start_skew * 1e6, 2),
            **prediction_fields(st.get("predicted_us_per_gen"), elapsed / steps * 1e6),
            "phases": phases,
            "per_rank": per_rank_block,
            "baseline_note": "reference publishes no numbers (BASELINE.md); vs_baseline is null",
        }
        if yard:
            out["yardstick_naive_byte_kernel"] = yard
            out["speedup_vs_yardstick"] = value / (yard["cell_updates_per_s"] * P)
        emit(out)
    if P > 1 or rccl is not None:
        import gc

        # Tear the engine (its graphs first) and then the RCCL communicator down on every rank while
        # all peers are still alive, not at interpreter exit where a rank could outlive its
        # neighbours.  (ncclCommDestroy while a graph that captured the communicator still exists
        # blocks: profiles/rccl_self_probe.txt.)
        sim.synchronize()
        del sim, transport, rccl
        gc.collect()
    if P > 1:
        import torch.distributed as dist

        dist.barrier(group=cpu_group)  # gloo: also fine when ranks share a GPU (rehearsal runs)
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

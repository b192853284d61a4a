"""The `gol` program on the HIP backend: multi-rank jobs oversubscribing one MI355X.

The reference maps rank r to GPU `r % deviceCount` (gol-with-cuda.cu:296), so `mpirun -n P` on one
GPU is its only multi-rank test rig.  Here P thread-ranks share device 0; RCCL needs
one rank per GPU, so the runtime stages halos through host memory (the same canonical-order
exchange, the same engine overlap/graph code).  Every dump is compared with the numpy torus oracle.
"""
import os
import subprocess

import numpy as np
import pytest

from gol_amd.ops import initial_board, numpy_step, quirk_model
from gol_amd.utils import read_dump

pytestmark = pytest.mark.gpu


def _run(gol_bin, args, cwd, nranks, env=None):
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "PMI_RANK", "PMI_SIZE"):
        e.pop(k, None)
    e.update(GOL_BACKEND="hip", GOL_NRANKS=str(nranks), GOL_VERBOSE="1")
    if env:
        e.update(env)
    return subprocess.run([gol_bin, *map(str, args)], cwd=cwd, env=e, capture_output=True, text=True, timeout=300)


def _board(cwd, P):
    parts = []
    for r in range(P):
        rank, first, cells = read_dump(os.path.join(cwd, f"Rank_{r}_of_{P}.txt"))
        parts.append((first, cells))
    parts.sort(key=lambda t: t[0])
    return np.vstack([c for _, c in parts])


@pytest.mark.parametrize(
    "P,env",
    [
        (2, {}),
        (3, {"GOL_HALO_DEPTH": "4"}),
        (4, {"GOL_OVERLAP": "0"}),
        (4, {"GOL_GRAPH": "0", "GOL_HALO_DEPTH": "3"}),
        (4, {"GOL_GLOBAL": "1", "GOL_DECOMP": "2d", "GOL_GRID": "2x2"}),
        (2, {"GOL_GLOBAL": "1", "GOL_DECOMP": "2d", "GOL_GRID": "2x1", "GOL_OVERLAP": "0"}),
        (3, {"GOL_WATCHDOG": "60"}),
        (3, {"GOL_SCHEDULE": "full"}),
        (2, {"GOL_SCHEDULE": "split", "GOL_KERNEL": "tile"}),
        (4, {"GOL_SCHEDULE": "split", "GOL_GLOBAL": "1", "GOL_DECOMP": "2d", "GOL_GRID": "2x2"}),
    ],
)
def test_threads_on_one_gpu_vs_oracle(gol_bin, tmp_path, P, env):
    N, gens = 256, 45
    r = _run(gol_bin, [5, N, gens, 256, 1], tmp_path, P, env)
    assert r.returncode == 0, r.stderr
    glob = env.get("GOL_GLOBAL") == "1"
    ref = numpy_step(initial_board(5, N, P, not glob), gens)
    assert np.array_equal(_board(tmp_path, P), ref)


@pytest.mark.parametrize("P", [1, 2, 3])
def test_compat_mode_on_gpu(gol_bin, tmp_path, P):
    N, gens = 70, 6
    r = _run(gol_bin, [5, N, gens, 256, 1], tmp_path, P, {"GOL_COMPAT": "reference"})
    assert r.returncode == 0, r.stderr
    assert np.array_equal(_board(tmp_path, P), quirk_model(initial_board(5, N, P, True), P, gens))


def test_watchdog_hang_on_gpu(gol_bin, tmp_path):
    r = _run(gol_bin, [5, 512, 4000, 256, 0], tmp_path, 2, {"GOL_FAULT": "1:64:hang", "GOL_WATCHDOG": "2"})
    assert r.returncode == 4, r.stderr
    assert "watchdog: no progress" in r.stderr


@pytest.mark.parametrize("env", [{}, {"GOL_GLOBAL": "1", "GOL_DECOMP": "2d", "GOL_GRID": "2x2"}])
def test_tile_kernel_multi_rank(gol_bin, tmp_path, env):
    P, N, gens = 4, 256, 37
    r = _run(gol_bin, [5, N, gens, 256, 1], tmp_path, P, dict(env, GOL_KERNEL="tile", GOL_HALO_DEPTH="6"))
    assert r.returncode == 0, r.stderr
    glob = env.get("GOL_GLOBAL") == "1"
    assert np.array_equal(_board(tmp_path, P), numpy_step(initial_board(5, N, P, not glob), gens))


@pytest.mark.parametrize(
    "N,env",
    [
        (256, {"GOL_HALO_DEPTH": "32", "GOL_KERNEL_DEPTH": "8"}),
        (256, {"GOL_HALO_DEPTH": "24", "GOL_KERNEL_DEPTH": "5", "GOL_KERNEL": "tile"}),
        (200, {"GOL_HALO_DEPTH": "20", "GOL_KERNEL_DEPTH": "6", "GOL_SCHEDULE": "split"}),
        (200, {"GOL_HALO_DEPTH": "17", "GOL_KERNEL_DEPTH": "4", "GOL_SCHEDULE": "full", "GOL_GRAPH": "0"}),
        (130, {}),
    ],
)
def test_multipass_deep_halos(gol_bin, tmp_path, N, env):
    """1-D supersteps of R generations run as several kernel passes that also compute the ghost
    rows (one exchange per R generations); remainders and unaligned widths included."""
    P, gens = 3, 101
    r = _run(gol_bin, [5, N, gens, 256, 1], tmp_path, P, env)
    assert r.returncode == 0, r.stderr
    assert np.array_equal(_board(tmp_path, P), numpy_step(initial_board(5, N, P, True), gens))


@pytest.mark.parametrize(
    "N,P,grid,env",
    [
        (256, 4, "2x2", {"GOL_HALO_DEPTH": "32", "GOL_KERNEL_DEPTH": "8", "GOL_SCHEDULE": "split"}),
        (256, 4, "2x2", {"GOL_HALO_DEPTH": "63", "GOL_KERNEL_DEPTH": "8", "GOL_SCHEDULE": "full"}),
        (256, 2, "2x1", {"GOL_HALO_DEPTH": "24", "GOL_KERNEL_DEPTH": "6"}),
        (200, 4, "2x2", {"GOL_HALO_DEPTH": "20", "GOL_KERNEL_DEPTH": "4", "GOL_KERNEL": "tile"}),
        (384, 6, "3x2", {}),
    ],
)
def test_multipass_2d(gol_bin, tmp_path, N, P, grid, env):
    """2-D supersteps of R generations as several passes: earlier passes also compute the ghost
    rows and ghost words (one 8-message exchange per R generations)."""
    gens = 131
    e = dict(env, GOL_GLOBAL="1", GOL_DECOMP="2d", GOL_GRID=grid)
    r = _run(gol_bin, [5, N, gens, 256, 1], tmp_path, P, e)
    assert r.returncode == 0, r.stderr
    assert np.array_equal(_board(tmp_path, P), numpy_step(initial_board(5, N, P, False), gens))


@pytest.mark.parametrize(
    "N,P,env",
    [
        (256, 2, {}),
        (256, 3, {"GOL_SCHEDULE": "split"}),
        (256, 4, {"GOL_SCHEDULE": "full"}),
        (200, 3, {"GOL_SCHEDULE": "split", "GOL_HALO_DEPTH": "20", "GOL_KERNEL_DEPTH": "6"}),
        (256, 4, {"GOL_GLOBAL": "1", "GOL_DECOMP": "2d", "GOL_GRID": "2x2", "GOL_SCHEDULE": "split"}),
        (256, 4, {"GOL_GLOBAL": "1", "GOL_DECOMP": "2d", "GOL_GRID": "2x2", "GOL_SCHEDULE": "full"}),
        (384, 6, {"GOL_GLOBAL": "1", "GOL_DECOMP": "2d", "GOL_GRID": "3x2"}),
        (256, 2, {"GOL_KERNEL": "tile", "GOL_SCHEDULE": "split"}),
        (256, 3, {"GOL_WATCHDOG": "60", "GOL_SCHEDULE": "split"}),
    ],
)
def test_device_transport_emulated(gol_bin, tmp_path, N, P, env):
    """GOL_TRANSPORT=p2p: thread ranks on one GPU with RCCL's semantics (device buffers, stream-
    ordered rendezvous copies, per-peer FIFO matching) — the device-transport engine paths that the
    multi-GPU RCCL runs take (device halos, split schedule, 2-D pack/unpack, collective autotune)."""
    gens = 101
    r = _run(gol_bin, [5, N, gens, 256, 1], tmp_path, P, dict(env, GOL_TRANSPORT="p2p"))
    assert r.returncode == 0, r.stderr
    assert "p2p-emulation" in r.stderr  # GOL_VERBOSE describes the transport
    glob = env.get("GOL_GLOBAL") == "1"
    assert np.array_equal(_board(tmp_path, P), numpy_step(initial_board(5, N, P, not glob), gens))


@pytest.mark.parametrize("env", [{}, {"GOL_GLOBAL": "1", "GOL_DECOMP": "2d", "GOL_GRID": "4x2"}])
def test_eight_ranks_one_gpu(gol_bin, tmp_path, env):
    """8 ranks (the node size of the scaling runs) with the RCCL-semantics data plane."""
    P, N, gens = 8, 256, 70
    r = _run(gol_bin, [5, N, gens, 256, 1], tmp_path, P, dict(env, GOL_TRANSPORT="p2p"))
    assert r.returncode == 0, r.stderr
    glob = env.get("GOL_GLOBAL") == "1"
    assert np.array_equal(_board(tmp_path, P), numpy_step(initial_board(5, N, P, not glob), gens))


def test_profile_and_metrics_on_gpu(gol_bin, tmp_path):
    """GOL_PROFILE=1 per-phase event timing + GOL_METRICS_JSON on the HIP backend."""
    import json

    path = tmp_path / "m.json"
    r = _run(gol_bin, [5, 512, 64, 256, 0], tmp_path, 2,
             {"GOL_PROFILE": "1", "GOL_METRICS_JSON": str(path), "GOL_ROCTX": "1"})
    assert r.returncode == 0, r.stderr
    m = json.loads(path.read_text())
    assert m["backend"] == "hip" and m["t_compute_ms"] > 0 and m["t_exchange_ms"] >= 0
    assert m["kernel"] and m["schedule"] in ("split", "full")


@pytest.mark.parametrize("threads,waves", [(256, 4), (512, 8), (1024, 16), (100, 8)])
def test_threads_per_block_selects_tile_workgroup(gol_bin, tmp_path, threads, waves):
    """threadsPerBlock is the LDS tile kernel's workgroup size (T/64 waves); invalid -> default 8."""
    N, gens = 512, 37
    r = _run(gol_bin, [5, N, gens, threads, 1], tmp_path, 1, {"GOL_KERNEL": "tile"})
    assert r.returncode == 0, r.stderr
    assert f"tile workgroup {waves} waves" in r.stderr
    assert ("threadsPerBlock=100" in r.stderr) == (threads == 100)
    assert np.array_equal(_board(tmp_path, 1), numpy_step(initial_board(5, N, 1, True), gens))


def test_perf_smoke_8192(gol_bin, tmp_path):
    """SURVEY §4.3 perf smoke: 8192^2 x 1000 generations through the CLI, cell-updates/s above a floor.

    Measured 4.8-4.9e13/s on one MI355X with folded tiles (profiles/tile_fold_ab.txt; 4.3-4.7e13 with
    plain tiles across boxes); the floor (4e13) catches a fallback to a slow path (the yardstick byte
    kernel runs at ≈4e11), the loss of the folded tiles' autotune choice beyond box noise, and any
    larger regression of the tile kernel."""
    import re

    r = _run(gol_bin, [5, 8192, 1000, 512, 0], tmp_path, 1)
    assert r.returncode == 0, r.stderr
    m = re.match(r"TOTAL DURATION : ([0-9.]+), number of cell updates = (\d+)\n", r.stdout)
    assert m, r.stdout
    secs, updates = float(m.group(1)), int(m.group(2))
    assert updates == 8192 * 8192 * 1000
    assert updates / secs > 4e13, f"{updates / secs:.3e} cell-updates/s"

"""The `gol` executable keeps the reference contract (gol-main.c:30-146) byte for byte.

Runs the native binary on the CPU backend (GOL_BACKEND=cpu) so it works without a GPU; multi-rank
runs use thread mode (GOL_NRANKS), the torchrun-style TCP rendezvous, and mpirun (MPICH) when
available.
"""
import os
import shutil
import socket
import subprocess

import numpy as np
import pytest

from gol_amd.ops import initial_board, numpy_step, quirk_model
from gol_amd.utils import read_dump

USAGE = (
    "GOL requires 5 arguments: pattern number, sq size of the world and the number of itterations, "
    "threads per block and output-on-off e.g. ./gol 0 32 2 512 0 \n"
)
BANNER = "This is the Game of Life running in parallel on a GPU on multiple ranks.\n"


def run(gol_bin, args, cwd, env=None, nranks=None):
    e = dict(os.environ)
    e["GOL_BACKEND"] = "cpu"
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "PMI_RANK", "PMI_SIZE"):
        e.pop(k, None)
    if nranks:
        e["GOL_NRANKS"] = str(nranks)
    if env:
        e.update(env)
    return subprocess.run([gol_bin, *map(str, args)], cwd=cwd, env=e, capture_output=True, text=True, timeout=120)


def load_board(cwd, P):
    parts = []
    for r in range(P):
        rank, first, cells = read_dump(os.path.join(cwd, f"Rank_{r}_of_{P}.txt"))
        assert rank == r
        parts.append((first, cells))
    parts.sort(key=lambda t: t[0])
    return np.vstack([c for _, c in parts])


def test_usage(gol_bin, tmp_path):
    r = run(gol_bin, [1, 2, 3], tmp_path)
    assert r.returncode == 255 and r.stdout == USAGE


def test_unknown_pattern(gol_bin, tmp_path):
    r = run(gol_bin, [9, 8, 1, 64, 1], tmp_path)
    assert r.returncode == 255
    assert r.stdout == "Pattern 9 has not been implemented \n"
    # like the reference, the dump file was opened before the pattern check
    assert os.path.exists(tmp_path / "Rank_0_of_1.txt")


def test_report_lines(gol_bin, tmp_path):
    r = run(gol_bin, [5, 64, 10, 512, 0], tmp_path)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines(keepends=True)
    assert len(lines) == 2 and lines[1] == BANNER
    assert lines[0].startswith("TOTAL DURATION : ") and lines[0].endswith(", number of cell updates = 40960\n")
    assert not list(tmp_path.glob("Rank_*"))  # on_off != 1 writes nothing


@pytest.mark.parametrize("threads,warns", [(64, False), (1024, False), (100, True), (0, True), (2048, True)])
def test_threads_per_block_hint(gol_bin, tmp_path, threads, warns):
    """threadsPerBlock is a hint (survey Q6): invalid values warn on stderr, the run and stdout are unchanged."""
    r = run(gol_bin, [5, 64, 10, threads, 1], tmp_path)
    assert r.returncode == 0, r.stderr
    assert r.stdout.endswith(", number of cell updates = 40960\n" + BANNER)
    assert ("threadsPerBlock=%d" % threads in r.stderr) == warns
    _, _, cells = read_dump(os.path.join(tmp_path, "Rank_0_of_1.txt"))
    assert np.array_equal(cells, numpy_step(initial_board(5, 64, 1, True), 10))


def test_dump_bytes(gol_bin, tmp_path):
    r = run(gol_bin, [4, 6, 0, 64, 1], tmp_path)
    assert r.returncode == 0
    text = (tmp_path / "Rank_0_of_1.txt").read_text()
    expect = "#" * 25 + " FINAL WORLD IN RANK 0 IS " + "#" * 31 + "\n" + "Row  0: 1 1 0 0 0 1 \n"
    expect += "".join("Row  %d: 0 0 0 0 0 0 \n" % i for i in range(1, 6))
    assert text == expect


@pytest.mark.parametrize("pattern", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("P", [1, 2, 3, 4, 8])
def test_patterns_multi_rank_threads(gol_bin, tmp_path, pattern, P):
    N, gens = 140, 7
    r = run(gol_bin, [pattern, N, gens, 256, 1], tmp_path, nranks=P)
    assert r.returncode == 0, r.stderr
    assert r.stdout.endswith(f"number of cell updates = {P * N * N * gens}\n" + BANNER)
    got = load_board(tmp_path, P)
    assert np.array_equal(got, numpy_step(initial_board(pattern, N, P, True), gens))


@pytest.mark.parametrize("P", [1, 2, 3, 4])
def test_compat_reference_quirks(gol_bin, tmp_path, P):
    N, gens = 24, 9
    r = run(gol_bin, [5, N, gens, 64, 1], tmp_path, env={"GOL_COMPAT": "reference"}, nranks=P)
    assert r.returncode == 0, r.stderr
    got = load_board(tmp_path, P)
    assert np.array_equal(got, quirk_model(initial_board(5, N, P, True), P, gens))


@pytest.mark.parametrize("env", [{"GOL_DECOMP": "2d", "GOL_GRID": "2x2"}, {"GOL_GLOBAL": "1"},
                                 {"GOL_GLOBAL": "1", "GOL_DECOMP": "2d"}, {"GOL_HALO_DEPTH": "1"}])
def test_decompositions_identical_dumps(gol_bin, tmp_path, env):
    N, gens, P = 256, 12, 4
    r = run(gol_bin, [5, N, gens, 256, 1], tmp_path, env=env, nranks=P)
    assert r.returncode == 0, r.stderr
    got = load_board(tmp_path, P)
    per_rank = env.get("GOL_GLOBAL") != "1"
    assert np.array_equal(got, numpy_step(initial_board(5, N, P, per_rank), gens))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("P", [2, 3])
def test_torchrun_style_tcp(gol_bin, tmp_path, P):
    N, gens = 96, 10
    port = _free_port()
    procs = []
    for r in range(P):
        e = dict(os.environ, GOL_BACKEND="cpu", RANK=str(r), WORLD_SIZE=str(P), LOCAL_RANK=str(r),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([gol_bin, "5", str(N), str(gens), "256", "1"], cwd=tmp_path, env=e,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert outs[0][0].endswith(BANNER) and outs[1][0] == ""
    assert np.array_equal(load_board(tmp_path, P), numpy_step(initial_board(5, N, P, True), gens))


MPIRUN = shutil.which("mpirun", path="/opt/conda/bin")


@pytest.mark.skipif(MPIRUN is None, reason="no mpirun")
def test_mpirun_launch(gol_bin, tmp_path):
    N, gens, P = 64, 6, 2
    e = dict(os.environ, GOL_BACKEND="cpu")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        e.pop(k, None)
    r = subprocess.run([MPIRUN, "-n", str(P), gol_bin, "3", str(N), str(gens), "256", "1"], cwd=tmp_path, env=e,
                       capture_output=True, text=True, timeout=120)
    if r.returncode != 0 and "HYDU" in (r.stderr + r.stdout):
        pytest.skip("mpirun cannot launch in this sandbox: " + r.stderr[-200:])
    assert r.returncode == 0, r.stderr
    assert np.array_equal(load_board(tmp_path, P), numpy_step(initial_board(3, N, P, True), gens))


def test_checkpoint_restart(gol_bin, tmp_path):
    N, P = 128, 2
    a = tmp_path / "a"
    b = tmp_path / "b"
    a.mkdir()
    b.mkdir()
    r = run(gol_bin, [5, N, 20, 256, 1], a, nranks=P, env={"GOL_CHECKPOINT_EVERY": "8",
                                                          "GOL_CHECKPOINT_PATH": str(tmp_path / "ck")})
    assert r.returncode == 0, r.stderr
    # restart from the generation-16 snapshot and finish the same 20 generations
    r2 = run(gol_bin, [5, N, 20, 256, 1], b, nranks=P, env={"GOL_RESTART": str(tmp_path / "ck")})
    assert r2.returncode == 0, r2.stderr
    for q in range(P):
        assert (a / f"Rank_{q}_of_{P}.txt").read_text() == (b / f"Rank_{q}_of_{P}.txt").read_text()


@pytest.mark.parametrize("restart_env,P2", [({}, 1), ({}, 3), ({"GOL_DECOMP": "2d", "GOL_GRID": "3x2"}, 6)])
def test_checkpoint_any_decomposition(gol_bin, tmp_path, restart_env, P2):
    """A checkpoint is the global board: written by a 2x2 grid, resumed on 1 rank, 3 strips or a 3x2 grid."""
    N = 192
    a = tmp_path / "a"
    b = tmp_path / "b"
    a.mkdir()
    b.mkdir()
    ck = str(tmp_path / "ck")
    r = run(gol_bin, [5, N, 16, 256, 0], a, nranks=4, env={"GOL_GLOBAL": "1", "GOL_DECOMP": "2d", "GOL_GRID": "2x2",
                                                          "GOL_CHECKPOINT_EVERY": "8", "GOL_CHECKPOINT_PATH": ck})
    assert r.returncode == 0, r.stderr
    assert os.path.exists(ck + ".gol") and not os.path.exists(ck + ".gol.tmp")
    r2 = run(gol_bin, [5, N, 21, 256, 1], b, nranks=P2, env={"GOL_GLOBAL": "1", "GOL_RESTART": ck, **restart_env})
    assert r2.returncode == 0, r2.stderr
    # the restarted run did the remaining 5 generations
    assert r2.stdout.startswith("TOTAL DURATION") and f"number of cell updates = {N * N * 5}" in r2.stdout
    assert np.array_equal(load_board(b, P2), numpy_step(initial_board(5, N, 1, False), 21))


def test_checkpoint_rejects_other_board(gol_bin, tmp_path):
    ck = str(tmp_path / "ck")
    r = run(gol_bin, [5, 64, 8, 256, 0], tmp_path, env={"GOL_CHECKPOINT_EVERY": "8", "GOL_CHECKPOINT_PATH": ck})
    assert r.returncode == 0, r.stderr
    r2 = run(gol_bin, [5, 128, 8, 256, 0], tmp_path, env={"GOL_RESTART": ck})
    assert r2.returncode != 0 and "holds a 64x64 board" in r2.stderr


@pytest.mark.parametrize("grid,P", [("3x2", 6), ("2x4", 8), ("4x1", 4)])
def test_2d_dumps_point_to_point(gol_bin, tmp_path, grid, P):
    """2-D dumps: tile/strip overlaps routed point to point (strips cut across several tile rows)."""
    N, gens = 256, 9
    r = run(gol_bin, [5, N, gens, 256, 1], tmp_path, nranks=P,
            env={"GOL_GLOBAL": "1", "GOL_DECOMP": "2d", "GOL_GRID": grid})
    assert r.returncode == 0, r.stderr
    assert np.array_equal(load_board(tmp_path, P), numpy_step(initial_board(5, N, 1, False), gens))


def test_fault_injection_aborts_all_ranks(gol_bin, tmp_path):
    r = run(gol_bin, [5, 64, 40, 256, 0], tmp_path, nranks=3, env={"GOL_FAULT": "1:16"})
    assert r.returncode == 3
    assert "injected abort on rank 1" in r.stderr


def test_watchdog_ends_hung_thread_job(gol_bin, tmp_path):
    """A rank that hangs (GOL_FAULT mode 'hang') is detected by the progress watchdog (exit 4)."""
    r = run(gol_bin, [5, 64, 400, 256, 0], tmp_path, nranks=2,
            env={"GOL_FAULT": "1:16:hang", "GOL_WATCHDOG": "1"})
    assert r.returncode == 4, r.stderr
    assert "watchdog: no progress" in r.stderr


def _tcp_job(gol_bin, tmp_path, P, env, args=(5, 64, 400, 256, 0)):
    port = _free_port()
    procs = []
    for q in range(P):
        e = dict(os.environ, GOL_BACKEND="cpu", RANK=str(q), WORLD_SIZE=str(P), LOCAL_RANK=str(q),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **env)
        procs.append(subprocess.Popen([gol_bin, *map(str, args)], cwd=tmp_path, env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=60))
        except subprocess.TimeoutExpired:
            for x in procs:
                x.kill()
            pytest.fail("a rank hung: the failure was not propagated")
    return [p.returncode for p in procs], outs


def test_watchdog_multiprocess_hang(gol_bin, tmp_path):
    codes, outs = _tcp_job(gol_bin, tmp_path, 3, {"GOL_FAULT": "1:16:hang", "GOL_WATCHDOG": "2"})
    assert all(c != 0 for c in codes), (codes, outs)
    assert any("watchdog" in err for _, err in outs)


def test_crashed_peer_does_not_hang_job(gol_bin, tmp_path):
    """A rank that dies without telling anyone (mode 'exit'): the others fail instead of hanging."""
    codes, outs = _tcp_job(gol_bin, tmp_path, 3, {"GOL_FAULT": "2:8:exit", "GOL_WATCHDOG": "5"})
    assert codes[2] == 3
    assert all(c != 0 for c in codes), (codes, outs)


def test_roctx_ranges_enabled(gol_bin, tmp_path):
    """GOL_ROCTX=1 loads the roctx library and brackets phases; the run output is unchanged."""
    r = run(gol_bin, [4, 64, 10, 256, 1], tmp_path, env={"GOL_ROCTX": "1"})
    assert r.returncode == 0, r.stderr
    assert "no roctx library" not in r.stderr
    assert r.stdout.endswith(BANNER)


def test_metrics_json(gol_bin, tmp_path):
    """GOL_METRICS_JSON: machine-readable run metrics on rank 0 (stdout contract unchanged)."""
    import json

    path = tmp_path / "m.json"
    r = run(gol_bin, [5, 128, 40, 256, 0], tmp_path, nranks=2, env={"GOL_METRICS_JSON": str(path)})
    assert r.returncode == 0, r.stderr
    assert r.stdout.endswith(BANNER)
    m = json.loads(path.read_text())
    assert m["ranks"] == 2 and m["generations"] == 40 and m["board"] == [256, 128]
    assert m["cell_updates"] == 2 * 128 * 128 * 40 and m["cell_updates_per_sec"] > 0
    assert m["backend"] == "cpu" and m["exchanges"] > 0 and m["halo_depth"] >= 1

"""CPU backend + Python API: patterns, stepping, decomposition invariance, planner, I/O helpers."""
import threading

import numpy as np
import pytest

from gol_amd.ops import initial_board, numpy_step, pack_cells, random_board, unpack_words
from gol_amd.ops.oracle import random_word


def test_random_word_matches_native(gol):
    for args in [(1, 2, 3, 4), (0x5EED, 1000, 7, 512), (2**63 + 5, 0, 0, 1)]:
        assert gol.native.random_word(*args) == random_word(*args)


@pytest.mark.parametrize("pattern", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("N", [1, 5, 64, 137])
def test_init_patterns(gol, pattern, N):
    s = gol.Simulation(N, backend="cpu").init(pattern)
    assert np.array_equal(s.board(), initial_board(pattern, N, 1, True))


@pytest.mark.parametrize("N,depth", [(3, 1), (65, 4), (200, 8), (130, 64)])
def test_step_vs_numpy(gol, N, depth):
    gens = 19
    s = gol.Simulation(N, backend="cpu", halo_depth=depth).init(5, seed=N)
    s.step(gens)
    assert s.generation == gens
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, N), gens))


def test_known_physics(gol):
    N = 32
    b = np.zeros((N, N), np.uint8)
    b[5, 4:7] = 1  # blinker: period 2
    b[20:22, 20:22] = 1  # block: still life
    s = gol.Simulation(N, backend="cpu")
    s.init(0)
    s.set_board(b)
    s.step(2)
    assert np.array_equal(s.board(), b)
    g = np.zeros((N, N), np.uint8)
    g[1, 2] = g[2, 3] = g[3, 1] = g[3, 2] = g[3, 3] = 1  # glider returns after 4*N generations on an N x N torus
    s.set_board(g)
    s.step(4 * N)
    assert np.array_equal(s.board(), g)
    s.set_board(np.ones((N, N), np.uint8))  # all ones: every cell has 8 neighbours -> all die
    s.step(1)
    assert s.population() == 0


def _run_threads(gol, N, P, gens, **kw):
    ts = gol.parallel.thread_transports(P)
    boards, fps = [None] * P, [None] * P

    def worker(r):
        s = gol.Simulation(N, ts[r], backend="cpu", **kw).init(5, seed=99)
        s.step(gens)
        boards[r] = (s.geometry.row0, s.geometry.col0, s.board())
        fps[r] = s.fingerprint()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    dec = gol.parallel.decomposition(N, P, kw.get("global_mode", False), kw.get("decomp", "1d"), kw.get("grid", ""),
                                     kw.get("width", 0))
    full = np.zeros((dec.H, dec.W), np.uint8)
    for r0, c0, b in boards:
        full[r0 : r0 + b.shape[0], c0 : c0 + b.shape[1]] = b
    return full, fps


@pytest.mark.parametrize("P,kw", [(2, {}), (3, {"halo_depth": 3}), (4, {"decomp": "2d", "grid": "2x2", "global_mode": True}),
                                  (6, {"decomp": "2d", "grid": "3x2", "global_mode": True}),
                                  (2, {"decomp": "2d", "grid": "2x1", "global_mode": True})])
def test_thread_ranks(gol, P, kw):
    N, gens = 384, 21
    full, fps = _run_threads(gol, N, P, gens, **kw)
    per_rank = not kw.get("global_mode", False)
    assert np.array_equal(full, numpy_step(initial_board(5, N, P, per_rank, 99), gens))
    assert len(set(fps)) == 1


@pytest.mark.parametrize("P,kw", [(1, {"width": 200}), (3, {"width": 130}), (1, {"width": 64 * 5, "global_mode": True}),
                                  (4, {"width": 64 * 6, "decomp": "2d", "grid": "2x2", "global_mode": True})])
def test_rectangular_boards(gol, P, kw):
    """Boards of N rows x `width` columns (per-rank strips or global boards) vs the numpy torus."""
    from gol_amd.ops.oracle import random_board

    N, gens = 96, 13
    full, fps = _run_threads(gol, N, P, gens, **kw)
    H = N if kw.get("global_mode") else N * P
    assert full.shape == (H, kw["width"])
    assert np.array_equal(full, numpy_step(random_board(H, kw["width"], 99), gens))
    assert len(set(fps)) == 1


@pytest.mark.parametrize("P,kw,depth", [
    (1, {"width": 128}, 32),                                                   # one rank: 32
    (2, {"width": 128, "global_mode": True}, 128),                             # 1-D strips of 2048 rows with neighbours
    (4, {"width": 256, "decomp": "2d", "grid": "2x2", "global_mode": True}, 56),  # 2-D tiles of 2048 rows: <= 63
    (2, {"width": 128, "global_mode": True, "halo_depth": 20}, 20),            # explicit depth wins
])
def test_auto_halo_depth(gol, P, kw, depth):
    """The auto halo depth (generations per exchange) is decided from rank-invariant inputs: 32 on one
    rank, 128 for 1-D strips of >= 2048 rows with neighbours, 56 for 2-D tiles of >= 2048 rows."""
    N = 4096
    ts = gol.parallel.thread_transports(P)
    got = [None] * P

    def worker(r):
        s = gol.Simulation(N, ts[r], backend="cpu", **kw).init(5, seed=1)
        got[r] = s.stats()["depth"]

    th = [threading.Thread(target=worker, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert got == [depth] * P, got


def test_fingerprint_decomposition_invariant(gol):
    N, gens = 256, 30
    one = gol.Simulation(N, backend="cpu", global_mode=True).init(5, 99).step(gens).fingerprint()
    _, fps = _run_threads(gol, N, 4, gens, global_mode=True, decomp="2d", grid="2x2")
    assert fps[0] == one


def test_bitpack_roundtrip():
    rng = np.random.default_rng(1)
    for w in (1, 63, 64, 65, 200):
        b = (rng.random((5, w)) < 0.5).astype(np.uint8)
        assert np.array_equal(unpack_words(pack_cells(b), w), b)


def test_native_cpu_torus_step(gol):
    b = random_board(40, 100, 3)
    out = gol.ops.cpu_torus_step(pack_cells(b), 100, 7)
    assert np.array_equal(unpack_words(out, 100), numpy_step(b, 7))


def test_plan_coverage(gol):
    lanes, st = gol.ops.build_plan([(0, 100, 0, 300)], 300, 100, 13, 4, False)
    cover = np.zeros((100, 300), int)
    for row0, col, flags, nrows in lanes:
        if flags & 1:
            cover[row0 : row0 + nrows, col] += 1
    assert (cover == 1).all()
    assert st["out_words"] == 100 * 300


@pytest.mark.parametrize("nw,h,rows", [(128, 300, 139), (300, 100, 13), (7, 50, 12)])
def test_fold_plan(gol, nw, h, rows):
    # folded tiles (step_tile_fold): segments of <= 30 words packed into 32 lanes, lanes 32-63 of each
    # tile repeat lanes 0-31, and every output word is stored by exactly one lane of the first halves
    lanes, st = gol.ops.build_plan([(0, h, 0, nw)], nw, h, rows, 24, True, fold=True)
    tiles = lanes.reshape(-1, 64, 4)
    assert (tiles[:, :32] == tiles[:, 32:]).all()
    cover = np.zeros((h, nw), int)
    for row0, col, flags, nrows in tiles[:, :32].reshape(-1, 4):
        if flags & 1:
            cover[row0 : row0 + nrows, col] += 1
    assert (cover == 1).all()
    assert st["out_words"] == h * nw
    for t in tiles[:, :32]:  # each segment: a halo lane, <= 30 output words, a halo lane
        run = 0
        for f in t[:, 2] & 1:
            run = run + 1 if f else 0
            assert run <= 30
        assert not (t[0, 2] & 1) and not (t[31, 2] & 1)


def test_dump_format_helpers(gol):
    from gol_amd.utils import format_dump, read_dump

    cells = np.array([[1, 0, 1], [0, 0, 1]], np.uint8)
    text = format_dump(2, cells, 10)
    native = gol.native.dump_header(2) + gol.native.format_rows(pack_cells(cells), 3, 10).decode()
    assert text == native


def test_cuda_not_required(gol):
    # the CPU path must work in this container (no GPU)
    s = gol.Simulation(16, backend="cpu").init(1).step(1)
    assert s.population() == 0

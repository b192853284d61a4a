"""step_flow (csrc/src/hip/flow_kernel.hip): a superstep's passes as ONE dependency-driven launch of a
persistent grid (GOL_SCHEDULE=flow).  Boards after G generations against numpy (small boards), a
PyTorch fp32 conv2d torus step on cuda:0 (the headline 32768^2 path, the driver's 5 + 20 cut) and the
thread-rank transport (ghost rows from neighbours, extended regions in the later passes).
Rule: gol-with-cuda.cu:239-257; generation loop: gol-main.c:93-116."""
import threading

import numpy as np
import pytest

from gol_amd.ops import initial_board, numpy_step, random_board, torch_step

pytestmark = pytest.mark.gpu


def _sim(gol, N, monkeypatch, **kw):
    monkeypatch.setenv("GOL_SCHEDULE", "flow")
    kw.setdefault("backend", "hip")
    kw.setdefault("device", 0)
    kw.setdefault("schedule", "flow")
    return gol.Simulation(N, **kw)


@pytest.mark.parametrize("N,gens,R", [(64, 1, 32), (64, 29, 32), (256, 40, 32), (512, 77, 32), (1024, 50, 64),
                                      (2048, 133, 128), (768, 20, 128)])
def test_flow_vs_numpy(gol, monkeypatch, N, gens, R):
    s = _sim(gol, N, monkeypatch, halo_depth=R).init(5, seed=N + gens)
    st = s.stats()
    assert "+flow" in st["schedule"], st
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, N + gens), gens))


def test_flow_rectangular_and_repeated(gol, monkeypatch):
    N, W = 300, 1024
    s = _sim(gol, N, monkeypatch, width=W).init(5, seed=3)
    ref = random_board(N, W, 3)
    for g in (24, 5, 48, 1, 30, 7):
        s.step(g)
        ref = numpy_step(ref, g)
        assert np.array_equal(s.board(), ref), g


@pytest.mark.parametrize("kmax", ["3", "5"])
def test_flow_shallow_cuts(gol, monkeypatch, kmax):
    """Cuts of shallow passes (more passes per launch: longer dependency chains)."""
    monkeypatch.setenv("GOL_FLOW_KMAX", kmax)
    N = 512
    s = _sim(gol, N, monkeypatch, halo_depth=32).init(5, seed=7)
    s.step(70)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, 7), 70))


def test_flow_headline_vs_torch(gol, monkeypatch):
    """The driver's bench path on the flow schedule: 32768^2, run hint 20, 5 + 20 generations, then +125."""
    import torch

    N, seed = 32768, 0x5EED
    s = _sim(gol, N, monkeypatch, run_hint=20).init(5, seed=seed)
    ref = torch.as_tensor(initial_board(5, N, 1, True, seed), device="cuda:0")
    for g in (5, 20, 125):
        s.step(g)
        ref = torch_step(ref, g, device="cuda:0")
        got = s.board()
        want = ref.cpu().numpy()
        assert np.array_equal(got, want), f"after +{g}: {int((got != want).sum())} cells differ"


@pytest.mark.parametrize("sched", ["flow", "flow+ov"])
@pytest.mark.parametrize("P,R", [(2, 32), (3, 32), (2, 128)])
def test_flow_thread_ranks_ghost_rows(gol, monkeypatch, P, R, sched):
    """Ranks with neighbours: the exchange fills the ghost rows, then one flow launch runs the superstep
    (its earlier passes also computing the ghost rows the later ones read).  flow+ov: the exchange runs
    on the comm stream while the launch's interior items run; the band items wait for its device flag
    (RCCL-semantics transport: device buffers, stream-ordered)."""
    N = 384 if R == 32 else 768
    gens = R * 3 + 11
    monkeypatch.setenv("GOL_SCHEDULE", sched)
    ts = gol.parallel.p2p_thread_transports(P)
    out, errs = [None] * P, []

    def rank_main(r):
        try:
            s = gol.Simulation(N, ts[r], backend="hip", device=0, global_mode=True, halo_depth=R, overlap=False,
                               subtiles=0, schedule=sched)
            s.init(5, seed=21)
            assert s.stats()["schedule"].endswith("+" + sched), s.stats()
            s.step(gens)
            out[r] = (s.geometry.row0, s.board())
        except Exception as e:  # pragma: no cover - reported below
            errs.append(repr(e))

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    board = np.zeros((N, N), dtype=np.uint8)
    for r0, b in out:
        board[r0 : r0 + b.shape[0]] = b
    assert np.array_equal(board, numpy_step(initial_board(5, N, 1, True, 21), gens))


def test_flow_2d_thread_ranks(gol, monkeypatch):
    """2-D blocks (8 neighbours, ghost words computed by the earlier passes of a superstep)."""
    N, gens = 512, 70
    monkeypatch.setenv("GOL_SCHEDULE", "flow")
    ts = gol.parallel.p2p_thread_transports(4)
    out, errs = [None] * 4, []

    def rank_main(r):
        try:
            s = gol.Simulation(N, ts[r], backend="hip", device=0, global_mode=True, decomp="2d", halo_depth=24,
                               overlap=False, subtiles=0, schedule="flow")
            s.init(5, seed=5)
            s.step(gens)
            g = s.geometry
            out[r] = (g.row0, g.col0, s.board())
        except Exception as e:  # pragma: no cover - reported below
            errs.append(repr(e))

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    board = np.zeros((N, N), dtype=np.uint8)
    for r0, c0, b in out:
        board[r0 : r0 + b.shape[0], c0 : c0 + b.shape[1]] = b
    assert np.array_equal(board, numpy_step(initial_board(5, N, 1, True, 5), gens))


@pytest.mark.parametrize("N,gens,hint,env", [(1024, 200, 200, {}), (1024, 137, 137, {"GOL_TILE_FOLD": "1"}),
                                            (2048, 96, 96, {"GOL_TILE_INPLACE": "1", "GOL_TILE_FOLD": "0"}),
                                            (768, 75, 0, {})])
def test_flow_tiles_vs_numpy(gol, monkeypatch, N, gens, hint, env):
    """Flow supersteps of LDS tile items (the tile kernel's device code, one workgroup per item): the
    hinted run is one launch of tile passes (folded, double-buffered or in place)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    s = _sim(gol, N, monkeypatch, kernel="tile", run_hint=hint).init(5, seed=N + gens)
    st = s.stats()
    assert "+flow" in st["schedule"] and st["kernel"].startswith("flow"), st
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, N + gens), gens))


def test_flow_config2_vs_torch(gol, monkeypatch):
    """BASELINE config 2 on the flow schedule (auto kernel: tile items at 8192^2), 1000-generation hint."""
    import torch

    N, seed = 8192, 0x5EED
    s = _sim(gol, N, monkeypatch, run_hint=1000).init(5, seed=seed)
    ref = torch.as_tensor(initial_board(5, N, 1, True, seed), device="cuda:0")
    for g in (100, 37, 1000):
        s.step(g)
        ref = torch_step(ref, g, device="cuda:0")
        got = s.board()
        want = ref.cpu().numpy()
        assert np.array_equal(got, want), f"after +{g}: {int((got != want).sum())} cells differ"

"""step_pipe (csrc/src/hip/pipe_kernel.hip): level-pipelined workgroups, one loader wave and NW - 1
stages of L generations chained through LDS rings.  Boards after G generations against numpy (small
boards), a PyTorch fp32 conv2d torus step on cuda:0 (large ones) and the thread-rank transport (ghost
rows from neighbours).  Rule: gol-with-cuda.cu:239-257."""
import threading

import numpy as np
import pytest

from gol_amd.ops import initial_board, numpy_step, random_board, torch_step

pytestmark = pytest.mark.gpu


def _sim(gol, N, geo, monkeypatch, **kw):
    monkeypatch.setenv("GOL_PIPE", geo)
    kw.setdefault("backend", "hip")
    kw.setdefault("device", 0)
    kw.setdefault("kernel", "pipe")
    return gol.Simulation(N, **kw)


@pytest.mark.parametrize("N,gens,geo", [(64, 1, "9,3,2"), (64, 29, "9,3,2"), (256, 40, "9,3,2"), (512, 77, "13,2,1"),
                                        (640, 100, "9,2,2"), (1024, 50, "5,4,4"), (1024, 61, "7,3,2"),
                                        (2048, 45, "11,2,2"), (512, 33, "16,2,1"), (768, 48, "5,1,1")])
def test_pipe_vs_numpy(gol, monkeypatch, N, gens, geo):
    nw, L, _ = (int(x) for x in geo.split(","))
    s = _sim(gol, N, geo, monkeypatch).init(5, seed=N + gens)
    assert s.stats()["kernel"].startswith(f"pipe@{(nw - 1) * L}"), s.stats()
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, N + gens), gens))


def test_pipe_rectangular_and_repeated(gol, monkeypatch):
    N, W = 300, 1024
    s = _sim(gol, N, "9,3,2", monkeypatch, width=W).init(5, seed=3)
    ref = random_board(N, W, 3)
    for g in (24, 5, 48, 1, 30):
        s.step(g)
        ref = numpy_step(ref, g)
        assert np.array_equal(s.board(), ref), g


def test_pipe_8192_vs_torch(gol, monkeypatch):
    import torch

    N, seed = 8192, 0x5EED
    s = _sim(gol, N, "9,3,2", monkeypatch, run_hint=1000).init(5, seed=seed)
    ref = torch.as_tensor(initial_board(5, N, 1, True, seed), device="cuda:0")
    for g in (100, 37):
        s.step(g)
        ref = torch_step(ref, g, device="cuda:0")
        got = s.board()
        assert np.array_equal(got, ref.cpu().numpy()), f"{int((got != ref.cpu().numpy()).sum())} cells differ"


@pytest.mark.parametrize("P,R", [(2, 32), (3, 32), (2, 128)])
def test_pipe_thread_ranks_ghost_rows(gol, monkeypatch, P, R):
    """Ranks with neighbours: the loader reads the exchanged ghost rows (no wrap); a superstep of R
    generations runs as 24-deep step_pipe passes (the earlier ones also computing the ghost rows the
    later ones read) plus step_temporal passes for the rest."""
    N = 384 if R == 32 else 768
    gens = R * 3 + 11
    monkeypatch.setenv("GOL_PIPE", "9,3,2")
    ts = gol.parallel.p2p_thread_transports(P)
    out, errs = [None] * P, []

    def rank_main(r):
        try:
            s = gol.Simulation(N, ts[r], backend="hip", device=0, global_mode=True, halo_depth=R, kernel="pipe",
                               overlap=False, subtiles=0)
            s.init(5, seed=21)
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


def test_pipe_rejects_bad_geometry(gol, monkeypatch):
    with pytest.raises(Exception, match="GOL_PIPE"):
        _sim(gol, 256, "6,2,1", monkeypatch).init(5, seed=1)
    with pytest.raises(Exception, match="halo depth"):
        _sim(gol, 256, "16,4,1", monkeypatch).init(5, seed=1)

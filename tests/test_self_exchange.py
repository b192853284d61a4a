"""Self-exchange mode (GOL_SELF_EXCHANGE=1): directions whose neighbour is the rank itself go
through the transport (send to self, receive from self) instead of wrapping by addressing.

On one rank this drives every halo path of the multi-rank engine (1-D full-pitch row blocks, 2-D
packed regions with corners, deep supersteps with ghost-row recompute) through a real transport:
here the CPU engine over SelfTransport's loopback and thread ranks; on the GPU suite a 1-rank RCCL
communicator (tests/test_gpu_rccl.py).  Reference exchange being replaced: gol-main.c:97-111.
"""
import threading

import numpy as np
import pytest

from gol_amd.ops import initial_board, numpy_step


@pytest.mark.parametrize("decomp", ["1d", "2d"])
@pytest.mark.parametrize("N,depth", [(64, 1), (128, 8), (130, 13), (256, 32)])
def test_self_exchange_cpu(gol, decomp, N, depth):
    gens = 3 * depth + 5
    s = gol.Simulation(N, backend="cpu", halo_depth=depth, decomp=decomp, self_exchange=True).init(5, seed=N)
    items = s.engine.halo_items(depth)
    if decomp == "2d" and N % 64 == 0:
        assert len(items) == 8  # N, S, W, E and the four corners, all to rank 0
    else:
        assert len(items) == 2  # N and S row blocks
    assert all(sp == 0 and rp == 0 for (_, sp, rp) in [(i[0], i[1], i[2]) for i in items])
    s.step(gens)
    st = s.stats()
    assert st["exchanges"] >= 1 and st["halo_bytes"] > 0
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, N), gens))


def test_self_exchange_off_by_default(gol):
    s = gol.Simulation(128, backend="cpu", halo_depth=8).init(5, seed=1)
    assert s.engine.halo_items(8) == []
    s.step(20)
    assert s.stats()["exchanges"] == 0


@pytest.mark.parametrize("grid", ["1x2", "2x1"])
def test_self_exchange_threads(gol, grid):
    """Two thread ranks in a 1x2 / 2x1 grid: one direction pair goes to the other rank, the other
    (self) pair also through the mailbox transport."""
    N, P, gens = 128, 2, 29
    ts = gol.parallel.thread_transports(P)
    out = [None] * P
    errs = []

    def worker(r):
        try:
            s = gol.Simulation(N, ts[r], backend="cpu", halo_depth=7, decomp="2d", grid=grid, global_mode=True,
                               self_exchange=True).init(5, seed=3)
            s.step(gens)
            out[r] = (s.geometry.row0, s.geometry.col0, s.board())
        except Exception as e:  # pragma: no cover - surfaced below
            errs.append(e)

    th = [threading.Thread(target=worker, args=(r,)) for r in range(P)]
    [t.start() for t in th]
    [t.join(60) for t in th]
    assert not errs, errs
    full = np.zeros((N, N), np.uint8)
    for r0, c0, b in out:
        full[r0:r0 + b.shape[0], c0:c0 + b.shape[1]] = b
    assert np.array_equal(full, numpy_step(initial_board(5, N, 1, False, 3), gens))

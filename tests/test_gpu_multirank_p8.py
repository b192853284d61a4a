"""Every superstep schedule a multi-rank run can pick, at P = 8 ranks, on the driver's bench cut.

The driver's scaling bench (bench.py, 1/2/4/8 GPUs) runs 5 warmup generations, then ONE hinted run of
20 generations (run_hint=20) per rank.  Here 8 thread ranks share one GPU through the RCCL-semantics
transport (p2p emulation: device buffers, stream-ordered rendezvous copies, per-peer FIFO matching), each
rank a 1-D strip of a global torus with neighbours on both sides, and the global board after 5 + 20
generations must equal the numpy torus oracle bit for bit.  One case per kept schedule:

    full         exchange on the compute stream, then the passes
    split        exchange on the comm stream overlapped with the interior, then the bands
    subtiles     two half-tiles on two streams, exchange first
    subtiles+ov  half 0's interior runs while the exchange is in flight

(``full+graph`` -- the ``full`` superstep captured with its RCCL group -- needs a capturable transport,
i.e. real RCCL, one rank per GPU: it is checked through the 1-rank RCCL communicator in
test_gpu_rccl.py; its exchange calls and matching are ``full``'s.)  Reference loop: gol-main.c:84-116.
"""
import threading

import numpy as np
import pytest

from gol_amd.ops import numpy_step, random_board

pytestmark = pytest.mark.gpu

P, H, W, SEED = 8, 1024, 2048, 41

CASES = [
    ("full", dict(schedule="full", subtiles=0), "full"),
    ("split", dict(schedule="split", subtiles=0), "split"),
    ("subtiles", dict(subtiles=2, subtile_overlap=0, kernel="temporal"), "full+subtiles2"),
    ("subtiles+ov", dict(subtiles=2, subtile_overlap=1, kernel="temporal"), "full+subtiles2ov"),
]


@pytest.mark.parametrize("name,kw,want", CASES, ids=[c[0] for c in CASES])
def test_p8_bench_cut(gol, monkeypatch, name, kw, want):
    monkeypatch.setenv("GOL_GRAPH_RCCL", "0")
    monkeypatch.setenv("GOL_SPINUP_MS", "0")
    ts = gol.parallel.p2p_thread_transports(P)
    out, errs = [None] * P, []

    def rank_main(r):
        try:
            s = gol.Simulation(P * H, ts[r], backend="hip", device=0, global_mode=True, width=W, halo_depth=32,
                               run_hint=20, **kw)
            s.init(5, seed=SEED)
            st = s.stats()
            assert st["schedule"] == want, st
            s.step(5)
            s.step(20)
            out[r] = (s.geometry.row0, s.board(), s.stats())
        except Exception as e:  # pragma: no cover - reported below
            errs.append(f"rank {r}: {e!r}")

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    assert all(o is not None for o in out)
    board = np.zeros((P * H, W), dtype=np.uint8)
    for r0, b, st in out:
        assert b.shape == (H, W)
        assert st["exchanges"] >= 2 and st["generations"] == 25, st
        board[r0 : r0 + H] = b
    want_board = numpy_step(random_board(P * H, W, SEED), 25)
    assert np.array_equal(board, want_board), f"{int((board != want_board).sum())} cells differ"


def test_p8_schedule_confirm(gol, monkeypatch):
    """The init-time schedule timing's close call settled collectively on the run path (confirm_schedule,
    forced with GOL_SCHED_CONFIRM=2): every rank sets up the runner-up, predicts it, and keeps or undoes it
    on the max-over-ranks predictions, so all ranks end on ONE schedule; then the 5 + 20 cut is exact."""
    monkeypatch.setenv("GOL_GRAPH_RCCL", "0")
    monkeypatch.setenv("GOL_SPINUP_MS", "0")
    monkeypatch.setenv("GOL_SCHED_CONFIRM", "2")
    ts = gol.parallel.p2p_thread_transports(P)
    out, errs = [None] * P, []

    def rank_main(r):
        try:
            s = gol.Simulation(P * H, ts[r], backend="hip", device=0, global_mode=True, width=W, halo_depth=32,
                               run_hint=20, kernel="temporal")
            s.init(5, seed=SEED)
            s.step(5)
            s.step(20)
            out[r] = (s.geometry.row0, s.board(), s.stats())
        except Exception as e:  # pragma: no cover - reported below
            errs.append(f"rank {r}: {e!r}")

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    assert all(o is not None for o in out)
    scheds = {o[2]["schedule"] for o in out}
    assert len(scheds) == 1, scheds
    assert all(" confirm:" in o[2]["tuning"] for o in out), out[0][2]["tuning"]
    board = np.zeros((P * H, W), dtype=np.uint8)
    for r0, b, st in out:
        board[r0 : r0 + H] = b
    want_board = numpy_step(random_board(P * H, W, SEED), 25)
    assert np.array_equal(board, want_board), f"{int((board != want_board).sum())} cells differ"

"""Real RCCL data plane on one GPU: a 1-rank communicator with the engine's self-exchange mode.

Every direction whose neighbour is the rank itself is sent with ncclSend to rank 0 and received
with ncclRecv from rank 0 inside one ncclGroupStart/End per superstep, on the engine's streams —
the exact calls a multi-GPU job makes (rccl_transport.cpp), replacing the reference's per-generation
MPI_Irecv/Isend/Wait of one byte row (gol-main.c:97-111).  Each schedule (one tile full / split,
two sub-tiles, 2-D packed halos with corners, RCCL captured in hipGraphs) is checked bit for bit
against the numpy torus oracle.
"""
import numpy as np
import pytest

from gol_amd.ops import initial_board, numpy_step, random_board

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl(gol):
    """One 1-rank RCCL communicator shared by the module (communicator init costs seconds)."""
    gol.native.hip_set_device(0)
    t = gol.native.make_rccl_transport(gol.native.SelfTransport())
    assert t.size() == 1 and t.device_buffers() and t.name().startswith("rccl")
    yield t


def _run(gol, rccl, N, gens, seed, **kw):
    kw.setdefault("backend", "hip")
    kw.setdefault("device", 0)
    s = gol.Simulation(N, rccl, self_exchange=True, **kw).init(5, seed=seed)
    s.step(gens)
    st = s.stats()
    got = s.board()
    s.synchronize()
    return got, st


@pytest.mark.parametrize("schedule", ["full", "split"])
@pytest.mark.parametrize("R", [8, 32])
def test_rccl_self_1d(gol, rccl, schedule, R):
    N, gens = 1024, 3 * R + 5
    got, st = _run(gol, rccl, N, gens, R, halo_depth=R, schedule=schedule, subtiles=0)
    assert st["schedule"] == schedule and st["exchanges"] >= 3, st
    assert st["halo_bytes"] > 0
    assert np.array_equal(got, numpy_step(initial_board(5, N, 1, True, R), gens))


def test_rccl_self_auto_schedule(gol, rccl):
    """The collective schedule timing (barrier + max over ranks) also runs on a 1-rank communicator."""
    N, gens = 2048, 70
    got, st = _run(gol, rccl, N, gens, 5, halo_depth=32, subtiles=0)
    assert st["schedule"].split("+")[0] in ("full", "split"), st
    assert "sched:" in st["tuning"], st
    assert np.array_equal(got, numpy_step(initial_board(5, N, 1, True, 5), gens))


@pytest.mark.parametrize("overlap", [0, 1, -1])
@pytest.mark.parametrize("R,gens", [(32, 2 * 32 + 20), (16, 5 * 16 + 3)])
def test_rccl_self_subtiles(gol, rccl, R, gens, overlap):
    """Two sub-tiles per rank: the rank's north / south halos go through RCCL straight into the halves;
    the seam between the halves is read in place by each half's first pass.  overlap=1: half 0's
    first pass (but its band next to the north halo) runs while the RCCL exchange is in flight;
    -1: the init-time timing picks one."""
    N = 1024
    got, st = _run(gol, rccl, N, gens, 9, halo_depth=R, subtiles=2, run_hint=gens, subtile_overlap=overlap)
    want = {0: ("full+subtiles2",), 1: ("full+subtiles2ov",), -1: ("full+subtiles2", "full+subtiles2ov")}[overlap]
    assert st["schedule"] in want, st
    if overlap == -1:
        assert "sched:subtiles=" in st["tuning"] and "sched:subtiles+ov=" in st["tuning"], st
    assert st["exchanges"] >= gens // R, st
    assert np.array_equal(got, numpy_step(initial_board(5, N, 1, True, 9), gens))


@pytest.mark.parametrize("kernel", ["temporal", "tile"])
@pytest.mark.parametrize("R", [5, 16])
def test_rccl_self_2d(gol, rccl, kernel, R):
    """2-D halo layout on one rank: 8 packed messages (N, S, W, E + corners) per superstep,
    pack/unpack kernels around the RCCL group."""
    N, gens = 640, 3 * R + 2
    got, st = _run(gol, rccl, N, gens, R, halo_depth=R, decomp="2d", kernel=kernel)
    assert st["exchanges"] >= 3, st
    assert np.array_equal(got, numpy_step(initial_board(5, N, 1, True, R), gens))


@pytest.mark.parametrize("decomp", ["1d", "2d"])
def test_rccl_self_graph_capture(gol, rccl, decomp, monkeypatch):
    """RCCL groups captured into hipGraphs (GOL_GRAPH_RCCL=1) and replayed."""
    monkeypatch.setenv("GOL_GRAPH_RCCL", "1")
    N, gens = 512, 16 * 8 + 8 * 3 + 5
    got, st = _run(gol, rccl, N, gens, 17, halo_depth=8, decomp=decomp, subtiles=0)
    assert st["graph_launches"] >= 1, st
    assert np.array_equal(got, numpy_step(initial_board(5, N, 1, True, 17), gens))


@pytest.mark.parametrize("H,W,decomp", [(2304, 1024, "2d"), (2048, 1536, "1d")])
def test_rccl_self_auto_depth_rectangular(gol, rccl, H, W, decomp):
    """Rectangular per-rank tiles with the auto halo depth of a rank with neighbours (56 in 2-D,
    128 in 1-D for >= 2048 rows): every superstep's halos through RCCL."""
    gens = 2 * 128 + 9
    got, st = _run(gol, rccl, H, gens, 6, width=W, decomp=decomp)
    assert st["depth"] == (56 if decomp == "2d" else 128), st
    assert st["exchanges"] >= 2, st
    assert np.array_equal(got, numpy_step(random_board(H, W, 6), gens))


@pytest.mark.parametrize("register", ["1", "0"])
def test_rccl_registered_boards(gol, rccl, monkeypatch, register):
    """The boards registered with the communicator (ncclCommRegister, zero-copy halos) or not: exact
    both ways, and the stats say which path ran."""
    monkeypatch.setenv("GOL_RCCL_REGISTER", register)
    N, gens = 1024, 2 * 32 + 7
    got, st = _run(gol, rccl, N, gens, 9, halo_depth=32, schedule="full", subtiles=0)
    assert st["registered"] == (register == "1"), st
    assert np.array_equal(got, numpy_step(initial_board(5, N, 1, True, 9), gens))


@pytest.mark.parametrize("pipe,H,R,gens", [("11,2,1", 1024, 20, 3 * 20 + 7), ("11,2,1", 1024, 0, 20),
                                              ("9,2,1", 768, 0, 2 * 16 + 7)])
def test_rccl_self_split_pipe(gol, rccl, monkeypatch, pipe, H, R, gens):
    """The split schedule of a strip whose tuned kernel is step_pipe (GOL_KERNEL=pipe): its passes are cut
    from measured step_pipe / step_temporal costs, the interior of the first pass runs while the RCCL
    exchange is in flight; a one-pass superstep runs its bands after the exchange on the comm stream,
    concurrently with the interior, and leaves the streams to be joined by the next superstep or the
    readout.  Several supersteps (R=20) and one multi-pass superstep; GOL_GRAPH_RCCL=1 leaves split
    supersteps eager."""
    monkeypatch.setenv("GOL_PIPE", pipe)
    monkeypatch.setenv("GOL_GRAPH_RCCL", "1")
    W = 4096
    got, st = _run(gol, rccl, H, gens, 3, width=W, schedule="split", kernel="pipe", subtiles=0, run_hint=gens,
                   halo_depth=R)
    assert st["schedule"] == "split" and st["exchanges"] >= 1 and st["graph_launches"] == 0, st
    assert np.array_equal(got, numpy_step(random_board(H, W, 3), gens))


@pytest.mark.parametrize("W", [1000, 4032 + 7])
def test_rccl_self_split_unaligned_width(gol, rccl, W):
    """A width that is not a multiple of 64 on a strip that wraps E/W onto itself: after a one-pass split
    superstep the ghost columns are refilled from the first and last words of every row, so that refill
    must follow both the interior (compute stream) and the bands (comm stream) -- the bands then run on
    the compute stream after the exchange instead of beside the interior.  Supersteps of
    one step_temporal pass (R = K = 8) and a one-pass remainder."""
    H, R = 1024, 8
    gens = 3 * R + 5
    got, st = _run(gol, rccl, H, gens, 4, width=W, schedule="split", kernel="temporal", subtiles=0, halo_depth=R,
                   run_hint=gens)
    assert st["schedule"] == "split" and st["exchanges"] >= 3, st
    assert np.array_equal(got, numpy_step(random_board(H, W, 4), gens))


def test_rccl_split_capture_refused(gol, rccl, monkeypatch, capfd):
    """An exchange is never enqueued on a stream forked into a graph capture (an RCCL group captured that
    way crashed librccl, docs/PERFORMANCE.md §17): GOL_GRAPH_SPLIT=1 attempts to capture split supersteps,
    whose exchange runs on the comm stream; the guard refuses it before any RCCL call, the capture is
    abandoned and the supersteps run eagerly, exact."""
    monkeypatch.setenv("GOL_GRAPH_SPLIT", "1")
    monkeypatch.setenv("GOL_GRAPH_RCCL", "1")
    H, R = 1024, 8
    gens = 2 * R + 3
    got, st = _run(gol, rccl, H, gens, 5, schedule="split", kernel="temporal", subtiles=0, halo_depth=R,
                   run_hint=gens)
    err = capfd.readouterr().err
    assert "capture's origin stream refused" in err, err[-2000:]
    assert st["schedule"] == "split" and st["graph_launches"] == 0, st
    assert np.array_equal(got, numpy_step(initial_board(5, H, 1, True, 5), gens))


@pytest.mark.parametrize("decomp,subtiles", [("1d", -1), ("2d", 0)])
def test_rccl_schedule_confirm(gol, rccl, monkeypatch, decomp, subtiles):
    """The close call of the schedule timing settled on the real run() path (confirm_schedule): the runner-up
    is set up in full (sub-tile halves allocated or freed, graphs re-captured) and predicted on a snapshot of
    the board, then kept or undone.  GOL_SCHED_CONFIRM=2 confirms whatever the margin.  The board must
    survive both switches: exact against numpy after the run."""
    monkeypatch.setenv("GOL_SCHED_CONFIRM", "2")
    N, R = 1024, 32
    gens = R + 9
    kw = {} if subtiles < 0 else {"subtiles": subtiles}
    got, st = _run(gol, rccl, N, gens, 12, halo_depth=R, decomp=decomp, run_hint=gens, **kw)
    assert " confirm:" in st["tuning"], st
    assert st["predicted_us_per_gen"] > 0, st
    assert np.array_equal(got, numpy_step(initial_board(5, N, 1, True, 12), gens))


@pytest.mark.parametrize("int_first,mark,bands,vwait", [("0", "0", "1", "1"), ("1", "1", "1", "0"), ("0", "1", "0", "1"),
                                                       ("1", "0", "0", "0")])
@pytest.mark.parametrize("decomp", ["1d", "2d"])
def test_rccl_split_order_knobs(gol, rccl, monkeypatch, int_first, mark, bands, vwait, decomp):
    """The split superstep's host order, ready-event record and band stream as knobs (the defaults -- interior
    first, no record between the first two passes, the bands on the comm stream beside the interior -- run in
    every split test above): the exchange enqueued before the interior (GOL_SPLIT_INT_FIRST=0), the record
    after every first pass (GOL_FIRST_PASS_MARK=1), the bands on the compute stream (GOL_SPLIT_BANDS_COMM=0) and
    the compute stream waiting for the comm stream's bands by event instead of by value (GOL_SPLIT_VALUE_WAIT=0),
    in 1-D and 2-D, supersteps of two passes and a remainder -- exact either way."""
    monkeypatch.setenv("GOL_SPLIT_INT_FIRST", int_first)
    monkeypatch.setenv("GOL_FIRST_PASS_MARK", mark)
    monkeypatch.setenv("GOL_SPLIT_BANDS_COMM", bands)
    monkeypatch.setenv("GOL_SPLIT_VALUE_WAIT", vwait)
    N, R = 768, 24
    gens = 2 * R + 7
    got, st = _run(gol, rccl, N, gens, 21, halo_depth=R, kernel_depth=12, decomp=decomp, schedule="split",
                   subtiles=0, run_hint=gens)
    assert st["schedule"] == "split" and st["exchanges"] >= 2, st
    assert np.array_equal(got, numpy_step(initial_board(5, N, 1, True, 21), gens))

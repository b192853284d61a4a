"""HIP backend numerics: the gfx950 kernels vs independent fp32/numpy oracles.

Every test here runs the native HIP path (temporal kernel or LDS kernel); there is no silent
fallback — Simulation(backend="hip") raises when no device is present.
"""
import numpy as np
import pytest

from gol_amd.ops import initial_board, numpy_step, random_board, torch_step

pytestmark = pytest.mark.gpu


def _sim(gol, N, **kw):
    kw.setdefault("backend", "hip")
    kw.setdefault("device", 0)
    return gol.Simulation(N, **kw)


@pytest.mark.parametrize("N", [1, 2, 3, 63, 64, 65, 127, 137, 200, 1000])
def test_random_board_vs_numpy(gol, N):
    gens = 11
    s = _sim(gol, N, halo_depth=8).init(5, seed=N)
    s.step(gens)
    ref = numpy_step(initial_board(5, N, 1, True, N), gens)
    assert np.array_equal(s.board(), ref)


@pytest.mark.parametrize("depth", [1, 2, 3, 4, 5, 6, 7, 8, 12, 16])
def test_every_depth(gol, depth):
    N, gens = 192, 37
    s = _sim(gol, N, halo_depth=depth, kernel_depth=depth, kernel="temporal").init(5, seed=3)
    s.step(gens)
    assert s.stats()["depth"] == depth and s.stats()["kernel_depth"] == depth
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, 3), gens))


@pytest.mark.parametrize("rows,waves", [(1, 0), (7, 0), (0, 3), (0, 100000)])
def test_plan_shapes(gol, rows, waves):
    N, gens = 640, 20
    s = _sim(gol, N, halo_depth=8, rows_per_wave=rows, waves_target=waves).init(5, seed=5)
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, 5), gens))


def test_lds_kernel(gol):
    N, gens = 300, 9
    s = _sim(gol, N, kernel="lds").init(5, seed=9)
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, 9), gens))


@pytest.mark.parametrize("graph", [True, False])
def test_graph_replay(gol, graph):
    N, gens = 512, 8 * 40 + 5  # several graph launches plus an eager remainder
    # (a pass kernel: with GOL_KERNEL=auto this board runs the resident kernel, one launch per run)
    s = _sim(gol, N, halo_depth=8, graph=graph, kernel="temporal").init(5, seed=11)
    s.step(gens)
    if graph:
        assert s.stats()["graph_launches"] >= 1
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, 11), gens))


@pytest.mark.parametrize("N,R", [(640, 8), (1024, 16), (4096, 32), (2048, 128)])
def test_subtiles_single_rank(gol, N, R):
    """GOL_SUBTILES=2: two half-tiles on two streams with seam copies and the torus wrap between
    them; remainder supersteps and repeated run() calls (copy in / copy back) stay exact."""
    s = _sim(gol, N, halo_depth=R, kernel="temporal", subtiles=2).init(5, seed=N + R)
    assert "subtiles2" in s.stats()["schedule"], s.stats()
    total = 0
    for gens in (R * 5 + 3, 7, R * 2):
        s.step(gens)
        total += gens
        if gens == 7:  # a reader between runs syncs the canonical board; the halves stay current
            assert s.population() == int(numpy_step(initial_board(5, N, 1, True, N + R), total).sum())
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, N + R), total))
    cells = (np.random.default_rng(N).random((N, N)) < 0.3).astype(np.uint8)
    s.set_board(cells)  # a writer invalidates the halves: the next run() reloads them
    s.step(R + 1)
    assert np.array_equal(s.board(), numpy_step(cells, R + 1))


@pytest.mark.parametrize("overlap", [0, 1])
@pytest.mark.parametrize("P", [2, 3])
def test_subtiles_thread_ranks(gol, P, overlap):
    """Sub-tiles with neighbours: each rank's north / south halos go to its two halves through the
    RCCL-semantics transport (thread ranks sharing one GPU).  overlap=1: half 0's first pass runs,
    but for its band next to the north halo, while the exchange is in flight (GOL_SUBTILE_OVERLAP)."""
    import threading

    N, gens = 512, 16 * 4 + 5
    ts = gol.parallel.p2p_thread_transports(P)
    out, errs = [None] * P, []

    def rank_main(r):
        try:
            s = gol.Simulation(N, ts[r], backend="hip", device=0, global_mode=True, halo_depth=16,
                               kernel="temporal", subtiles=2, subtile_overlap=overlap)
            s.init(5, seed=17)
            assert s.stats()["schedule"].endswith({0: "+subtiles2", 1: "+subtiles2ov"}[overlap]), s.stats()
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
    ref = numpy_step(initial_board(5, N, 1, True, 17), gens)
    for r0, b in out:
        assert np.array_equal(b, ref[r0 : r0 + b.shape[0]])


def test_run_hint_single_graph(gol):
    """run_hint: one replay graph covers the whole expected run (37 supersteps here), other run
    lengths still use the 16/4/1 ladder; both parities stay exact."""
    N, R = 512, 8
    hint = R * 37 + 5
    s = _sim(gol, N, halo_depth=R, kernel_depth=R, kernel="temporal", run_hint=hint, subtiles=0).init(5, seed=13)
    g0 = s.stats()["graph_launches"]
    s.step(hint)
    assert s.stats()["graph_launches"] - g0 == 1, s.stats()
    s.step(R * 21 + 3)
    s.step(hint)
    total = 2 * hint + R * 21 + 3
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, 13), total))


@pytest.mark.parametrize("subtiles", [0, 2])
def test_run_hint_short_run(gol, subtiles):
    """A hinted run shorter than one superstep (the driver's bench: 20 generations, R = 64): one graph
    replay in the one-tile mode; eager in the sub-tile mode (graphs of its passes measured slower).
    Exact either way."""
    N, hint = 1024, 20
    s = _sim(gol, N, halo_depth=64, kernel="temporal", run_hint=hint, subtiles=subtiles).init(5, seed=23)
    assert ("+subtiles2" in s.stats()["schedule"]) == (subtiles == 2), s.stats()
    s.step(5)  # unhinted: eager
    g0 = s.stats()["graph_launches"]
    assert g0 == 0, s.stats()
    s.step(hint)
    assert s.stats()["graph_launches"] - g0 == (0 if subtiles else 1), s.stats()
    s.step(hint)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, 23), 5 + 2 * hint))


@pytest.mark.parametrize("N,R,gens", [(1024, 32, 200), (1088, 16, 77), (4096, 64, 150), (576, 8, 61)])
def test_subtiles_seam_reads(gol, N, R, gens):
    """Two sub-tiles: the first pass of every superstep reads the other half's edge rows and the
    torus wrap in place (STEP_SEAM), the passes rotate through three buffers; odd heights, remainder
    supersteps and several run() calls."""
    s = _sim(gol, N, halo_depth=R, kernel="temporal", subtiles=2).init(5, seed=N + R)
    assert s.stats()["schedule"].endswith("+subtiles2"), s.stats()  # no neighbours: no overlap variant
    s.step(gens // 3)
    s.step(gens - gens // 3)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, N + R), gens))


@pytest.mark.parametrize("R,K", [(16, 8), (8, 8), (24, 8)])
def test_graph_replay_after_parity_flip(gol, R, K):
    """Replays are keyed by buffer parity and track it: graphs of 16, 4 and 1 supersteps (1 or 3
    passes per superstep flip the parity per superstep) interleaved with eager remainders."""
    N = 512
    s = _sim(gol, N, halo_depth=R, kernel_depth=K, kernel="temporal", subtiles=0).init(5, seed=12)  # graphs
    total = 0
    for gens in (R * 16, 8, R * 21 + 3, 5, R * 16 + R * 4 + R + 7, 2 * R + 1):
        s.step(gens)
        total += gens
    assert s.stats()["graph_launches"] >= 6
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, 12), total))


def test_large_board_vs_torch_conv(gol):
    import torch

    N, gens = 4096, 30
    s = _sim(gol, N).init(5, seed=21)
    s.step(gens)
    ref = torch_step(random_board(N, N, 21), gens, device="cuda:0").cpu().numpy()
    assert np.array_equal(s.board(), ref)
    assert s.population() == int(ref.sum())


@pytest.mark.parametrize("pattern", [0, 1, 2, 3, 4])
def test_reference_patterns(gol, pattern):
    N, gens = 150, 6
    s = _sim(gol, N).init(pattern)
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(pattern, N, 1, True), gens))


def test_fingerprint_matches_cpu(gol):
    N, gens = 333, 17
    a = _sim(gol, N).init(5, seed=4).step(gens)
    b = gol.Simulation(N, backend="cpu").init(5, seed=4).step(gens)
    assert a.fingerprint() == b.fingerprint() and a.population() == b.population()


def test_set_board_roundtrip(gol):
    N = 129
    s = _sim(gol, N).init(0)
    cells = (np.random.default_rng(0).random((N, N)) < 0.4).astype(np.uint8)
    s.set_board(cells)
    assert np.array_equal(s.board(), cells)
    s.step(5)
    assert np.array_equal(s.board(), numpy_step(cells, 5))


def test_naive_yardstick(gol):
    t, pop = gol.native.naive_byte_run(256, 10, 256, True, 0x5EED)
    assert t > 0
    assert pop == int(numpy_step(random_board(256, 256, 0x5EED), 10).sum())


@pytest.mark.parametrize("depth", [6, 7, 12])
def test_pingpong_loop_depths(gol, depth):
    """Depths that run the two-triple steady loop (K = 6, 7, 12), with tall segments (300 rows) so the
    loop runs many six-row iterations plus its leftover triple and tail rows, on the torus and with
    ghost rows (two passes per superstep)."""
    N = 2048
    for R, gens in ((depth, 3 * depth + 1), (2 * depth, 2 * depth + 5)):
        s = _sim(gol, N, halo_depth=R, kernel_depth=depth, kernel="temporal", rows_per_wave=300, subtiles=0)
        s.init(5, seed=depth + R)
        s.step(gens)
        assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, depth + R), gens)), (depth, R)


@pytest.mark.parametrize("depth", [1, 3, 5, 7, 8, 16])
def test_kernel_depth_passes(gol, depth):
    """Every instantiated temporal depth as the pass depth, with multi-pass supersteps of 2*depth+1
    generations (balanced pass cuts) and an odd remainder."""
    N, gens = 700, 7 * depth + 5
    s = _sim(gol, N, halo_depth=min(64, 2 * depth + 1), kernel_depth=depth, kernel="temporal").init(5, seed=depth)
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, depth), gens))


@pytest.mark.parametrize("graph", [True, False])
def test_watchdog_fenced_run(gol, graph):
    """Watchdog mode bounds the host lookahead with polled events; results are unchanged."""
    N, gens = 512, 8 * 40 + 3
    s = _sim(gol, N, halo_depth=8, graph=graph, watchdog=60.0).init(5, seed=21)
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, 21), gens))


@pytest.mark.parametrize("tile_waves", [4, 8, 16])
@pytest.mark.parametrize("depth", [1, 2, 5, 8, 13])
def test_tile_kernel_depths(gol, tile_waves, depth):
    """LDS-resident temporal kernel (any runtime depth) vs numpy."""
    N, gens = 700, 3 * depth + 5
    s = _sim(gol, N, halo_depth=depth, kernel_depth=depth, kernel="tile", tile_waves=tile_waves).init(5, seed=depth)
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, depth), gens))


@pytest.mark.parametrize("N", [1, 3, 65, 137, 1000, 4096])
def test_tile_kernel_sizes(gol, N):
    gens = 29
    s = _sim(gol, N, halo_depth=8, kernel="tile").init(5, seed=N + 1)
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, N + 1), gens))


@pytest.mark.parametrize("fold", ["0", "1"])
@pytest.mark.parametrize("N,depth,tile_waves", [(2048, 24, 8), (700, 13, 16), (1000, 5, 4), (640, 32, 8)])
def test_tile_fold(gol, monkeypatch, fold, N, depth, tile_waves):
    """Folded tiles (GOL_TILE_FOLD=1: 32-lane tiles twice as tall, lanes 32-63 streaming the bottom
    half upwards, mirrored middle rows) and plain tiles (0) vs numpy, odd and even tile heights."""
    monkeypatch.setenv("GOL_TILE_FOLD", fold)
    gens = 2 * depth + 3
    s = _sim(gol, N, halo_depth=depth, kernel_depth=depth, kernel="tile", tile_waves=tile_waves).init(5, seed=N + depth)
    assert ("tile_plan=fold," in s.stats()["tuning"]) == (fold == "1"), s.stats()["tuning"]
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, N + depth), gens))


@pytest.mark.parametrize("N,depth,tile_waves", [(2048, 24, 8), (1100, 9, 16)])
def test_tile_fold_inplace(gol, monkeypatch, N, depth, tile_waves):
    """Folded tiles updated in place (GOL_TILE_FOLD=1, GOL_TILE_INPLACE=1: side-row copies, mirrored
    middle rows read from the copy) vs numpy."""
    monkeypatch.setenv("GOL_TILE_FOLD", "1")
    monkeypatch.setenv("GOL_TILE_INPLACE", "1")
    gens = 2 * depth + 5
    s = _sim(gol, N, halo_depth=depth, kernel_depth=depth, kernel="tile", tile_waves=tile_waves).init(5, seed=N)
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, N), gens))


@pytest.mark.parametrize("fold", ["0", "1"])
def test_tile_fold_split_ghost_rows(gol, monkeypatch, fold):
    """Folded tiles in the split schedule (interior and boundary regions, ghost rows, no y-wrap)."""
    monkeypatch.setenv("GOL_TILE_FOLD", fold)
    N, gens = 1024, 8 * 6 + 5
    s = _sim(gol, N, halo_depth=8, kernel="tile", force_split=True).init(5, seed=41)
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, 41), gens))


@pytest.mark.parametrize("rows", [1, 5, 64])
def test_tile_kernel_plan_rows(gol, rows):
    N, gens = 640, 21
    s = _sim(gol, N, halo_depth=6, kernel="tile", rows_per_wave=rows).init(5, seed=77)
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, 77), gens))


@pytest.mark.parametrize("N", [96, 2048])
def test_auto_kernel_choice(gol, N):
    """GOL_KERNEL=auto times the candidate kernels at init (pass kernels, and on boards without
    neighbours the resident kernel) and keeps one; results are exact either way."""
    gens = 53
    s = _sim(gol, N, halo_depth=8, kernel="auto").init(5, seed=N)
    k = s.stats()["kernel"]
    assert k in ("temporal", "tile") or k.startswith("resident@") or k.startswith("pipe@"), k
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, N), gens))


@pytest.mark.parametrize("N", [1000, 8192])
def test_auto_single_rank_depth_32(gol, N):
    """One rank, auto depth (32): the tuner may pick tile passes of 24 or 32 generations (not a
    register-kernel depth); remainder supersteps and every pass cut stay exact."""
    gens = 32 * 5 + 8 + 3
    s = _sim(gol, N, kernel="auto").init(5, seed=N + 1)
    st = s.stats()
    assert st["depth"] == 32 and st["kernel"] in ("temporal", "tile"), st
    if st["kernel"] == "temporal":
        assert st["kernel_depth"] <= 16, st
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, N + 1), gens))


@pytest.mark.parametrize("kernel", ["temporal", "tile"])
@pytest.mark.parametrize("graph", [True, False])
def test_forced_split_schedule(gol, kernel, graph):
    """Interior on the compute stream + boundary bands after the (empty) comm-stream exchange
    (the multi-GPU split schedule, forced on one rank) is exact."""
    N, gens = 1024, 8 * 36 + 5
    s = _sim(gol, N, halo_depth=8, kernel=kernel, graph=graph, force_split=True)
    s.init(5, seed=31)
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, 31), gens))


@pytest.mark.parametrize("R,K", [(32, 8), (24, 6), (13, 4)])
def test_single_rank_multipass(gol, R, K):
    N, gens = 512, 3 * R + 7
    s = _sim(gol, N, halo_depth=R, kernel_depth=K).init(5, seed=R)
    assert s.stats()["depth"] == R and s.stats()["kernel_depth"] <= K
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, R), gens))


@pytest.mark.parametrize("decomp,grid,P", [("1d", "", 3), ("2d", "2x2", 4)])
def test_python_threads_device_transport(gol, decomp, grid, P):
    """Simulation API, one Python thread per rank, RCCL-semantics transport on one GPU."""
    import threading

    N, gens = 256, 77
    ts = gol.parallel.p2p_thread_transports(P)
    out, errs = [None] * P, []

    def rank_main(r):
        try:
            s = gol.Simulation(N, ts[r], backend="hip", device=0, global_mode=True, decomp=decomp, grid=grid)
            s.init(5, seed=9)
            s.step(gens)
            out[r] = (s.geometry.row0, s.geometry.col0, s.board())
        except Exception as e:  # pragma: no cover - reported below
            errs.append(repr(e))

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    board = np.zeros((N, N), dtype=np.uint8)
    for r0, c0, b in out:
        board[r0 : r0 + b.shape[0], c0 : c0 + b.shape[1]] = b
    assert np.array_equal(board, numpy_step(initial_board(5, N, 1, True, 9), gens))


def test_threads_device_transport_deep_halo_128(gol):
    """Tall 1-D strips (>= 2048 rows) get the auto halo depth 128: 16 kernel passes per exchange,
    the earlier ones also computing ghost rows.  2 thread ranks on one GPU (RCCL-semantics
    transport), 16384^2 board vs the PyTorch conv2d oracle."""
    import threading

    import torch

    N, P, gens = 16384, 2, 128 + 64 + 13
    ts = gol.parallel.p2p_thread_transports(P)
    out, errs = [None] * P, []

    def rank_main(r):
        try:
            s = gol.Simulation(N, ts[r], backend="hip", device=0, global_mode=True)
            s.init(5, seed=5)
            assert s.stats()["depth"] == 128, s.stats()
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
    ref = torch_step(random_board(N, N, 5), gens, device="cuda:0").cpu().numpy()
    for r0, b in out:
        assert np.array_equal(b, ref[r0 : r0 + b.shape[0]])
    del ref
    torch.cuda.empty_cache()


@pytest.mark.parametrize("kernel", ["temporal", "tile"])
def test_known_physics_gpu(gol, kernel):
    """Blinker period 2, block still life, glider back home after 4N generations on an N x N torus,
    all-ones board dies in one generation — on the HIP kernels."""
    N = 128
    s = _sim(gol, N, kernel=kernel).init(0)
    b = np.zeros((N, N), np.uint8)
    b[5, 4:7] = 1
    b[60:62, 60:62] = 1
    s.set_board(b)
    s.step(2)
    assert np.array_equal(s.board(), b)
    g = np.zeros((N, N), np.uint8)
    g[1, 2] = g[2, 3] = g[3, 1] = g[3, 2] = g[3, 3] = 1
    s.set_board(g)
    s.step(4 * N)
    assert np.array_equal(s.board(), g)
    s.set_board(np.ones((N, N), np.uint8))
    s.step(1)
    assert s.population() == 0


@pytest.mark.parametrize("H,W,kernel", [(300, 1000, "temporal"), (130, 4096, "tile"), (2048, 192, "auto"),
                                        (517, 333, "temporal")])
def test_rectangular_boards(gol, H, W, kernel):
    """N rows x width columns (the per-rank tiles of multi-GPU configs, measured on one GPU)."""
    gens = 29
    s = _sim(gol, H, width=W, kernel=kernel).init(5, seed=H)
    s.step(gens)
    assert s.board().shape == (H, W)
    assert np.array_equal(s.board(), numpy_step(random_board(H, W, H), gens))


@pytest.mark.parametrize("inplace", ["0", "1"])
@pytest.mark.parametrize("levels", ["1", "2", "4"])
@pytest.mark.parametrize("tile_waves", [4, 8, 16])
def test_tile_variants(gol, monkeypatch, inplace, levels, tile_waves):
    """Tile kernel: double-buffered or in place (private halo copies), 1/2/4 generations per LDS
    pass, every workgroup size; depth 13 leaves a pass of each smaller level count."""
    monkeypatch.setenv("GOL_TILE_INPLACE", inplace)
    monkeypatch.setenv("GOL_TILE_LEVELS", levels)
    N, gens = 700, 13 * 3 + 5
    s = _sim(gol, N, kernel="tile", halo_depth=13, kernel_depth=13, tile_waves=tile_waves).init(5, seed=21)
    s.step(gens)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, 21), gens))


def test_tile_inplace_auto_tall_tiles(gol):
    """A board whose one-round tiles exceed the double buffer: the planner switches to the in-place
    tile (one round of ~137-row tiles at 4096 x 32768), checked against the torch oracle."""
    import torch

    H, W, gens = 4096, 32768, 64
    s = _sim(gol, H, width=W, kernel="tile", kernel_depth=32).init(5, seed=4)
    s.step(gens)
    ref = torch_step(random_board(H, W, 4), gens, device="cuda").cpu().numpy()
    assert np.array_equal(s.board(), ref)
    del torch


def test_checkpoint_across_decompositions_hip(gol, tmp_path):
    """A HIP engine's checkpoint (one global board file) resumed by 2 thread ranks in a 2x1 grid on
    the CPU backend: the file depends on neither the decomposition nor the backend."""
    import threading

    N, g1, g2 = 512, 40, 23
    prefix = str(tmp_path / "ck")
    a = _sim(gol, N, global_mode=True).init(5, seed=8)
    a.step(g1)
    a.checkpoint(prefix)
    ts = gol.parallel.thread_transports(2)
    parts = [None, None]

    def rank(r):
        b = gol.Simulation(N, ts[r], backend="cpu", global_mode=True, decomp="2d", grid="2x1").init(0)
        assert b.restore(prefix) == g1
        b.step(g2)
        parts[r] = (b.geometry.col0, b.board())

    th = [threading.Thread(target=rank, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    full = np.hstack([p[1] for p in sorted(parts, key=lambda p: p[0])])
    assert np.array_equal(full, numpy_step(initial_board(5, N, 1, False, 8), g1 + g2))


@pytest.mark.parametrize("N,R", [(385, 64), (388, 64), (259, 43)])
def test_uneven_strips_collective_schedule(gol, N, R):
    """Strips of 129/128/128 rows with R = 64 (and neighbours of it): whether the split schedule is
    possible is decided from the smallest strip on every rank, so the collective schedule timing is
    entered by all ranks or none (a per-rank decision would hang or mismatch the exchanges)."""
    import threading

    P, gens = 3, 2 * R + 11
    ts = gol.parallel.p2p_thread_transports(P)
    out, errs = [None] * P, []

    def rank_main(r):
        try:
            s = gol.Simulation(N, ts[r], backend="hip", device=0, global_mode=True, halo_depth=R, width=320)
            s.init(5, seed=31)
            s.step(gens)
            out[r] = (s.geometry.row0, s.board(), s.stats()["schedule"])
        except Exception as e:  # pragma: no cover - reported below
            errs.append(repr(e))

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    assert len({o[2] for o in out}) == 1, [o[2] for o in out]  # one schedule on every rank
    board = np.vstack([b for _, b, _ in sorted(out, key=lambda o: o[0])])
    assert np.array_equal(board, numpy_step(random_board(N, 320, 31), gens))


def test_multi_round_plans(gol, monkeypatch):
    """Streaming plans of several rounds (plan.hpp round_balanced_rows, big tiles by default), forced on a
    16384^2 board by a tiny segment target (GOL_ROUND_ROWS_PER_LEVEL=1, read when the engine is built):
    the plan must hold more waves than the one-round plan, and the board must match a torch oracle."""
    import torch

    N, gens, seed = 16384, 8 * 3 + 5, 21
    one = _sim(gol, N, halo_depth=8, kernel="temporal", subtiles=False).init(5, seed=seed)
    waves1 = one.stats()["plan_waves"]
    del one
    monkeypatch.setenv("GOL_ROUND_ROWS_PER_LEVEL", "1")
    s = _sim(gol, N, halo_depth=8, kernel="temporal", subtiles=False).init(5, seed=seed)
    assert s.stats()["plan_waves"] > waves1
    s.step(gens)
    ref = torch_step(torch.as_tensor(initial_board(5, N, 1, True, seed), device="cuda:0"), gens, device="cuda:0")
    assert np.array_equal(s.board(), ref.cpu().numpy())


def test_torch_device_sync_covers_engine_streams(gol):
    """bench.py ends the timed run with torch.cuda.synchronize() alone: hipDeviceSynchronize must wait for
    the engine's own non-blocking streams (both sub-tile halves at 32768^2)."""
    import torch

    torch.cuda.synchronize()
    s = _sim(gol, 32768).init(5, seed=2)
    s.step(8)
    s.synchronize()
    assert s.engine.gpu_idle()
    s.step(1000)  # ~10 ms of GPU work, enqueued in well under that
    torch.cuda.synchronize()
    assert s.engine.gpu_idle()


@pytest.mark.parametrize("subtiles", [0, 2])
def test_prediction_without_snapshot(gol, monkeypatch, subtiles):
    """predict_run's scratch-state branch (no memory for a board snapshot, as on BASELINE config 5's 2^20-row
    tile; forced with GOL_PREDICT_SNAPSHOT=0): the prediction is measured and the board stays intact, so
    the hinted run after init is exact."""
    monkeypatch.setenv("GOL_PREDICT_SNAPSHOT", "0")
    N, hint = 2048, 20
    s = _sim(gol, N, halo_depth=64, kernel="temporal", run_hint=hint, subtiles=subtiles).init(5, seed=31)
    st = s.stats()
    assert st["predicted_us_per_gen"] > 0 and st["predicted_gens"] == hint, st
    s.step(5)
    s.step(hint)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, 31), 5 + hint))

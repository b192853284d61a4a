"""The resident kernel (step_resident, csrc/src/hip/resident_kernel.hip): a whole run in one launch,
tiles kept in registers, K-deep halos exchanged between workgroups inside the kernel.  Boards after
G generations are compared with numpy (small boards) or a PyTorch fp32 conv2d torus step on cuda:0
(BASELINE config 2, 8192^2).  Rule: gol-with-cuda.cu:239-257."""
import numpy as np
import pytest

from gol_amd.ops import initial_board, numpy_step, torch_step

pytestmark = pytest.mark.gpu


def _sim(gol, N, **kw):
    kw.setdefault("backend", "hip")
    kw.setdefault("device", 0)
    kw.setdefault("kernel", "resident")
    return gol.Simulation(N, **kw)


@pytest.mark.parametrize("N,gens,kin", [(64, 1, 8), (64, 37, 8), (128, 40, 16), (256, 100, 12), (640, 57, 24),
                                        (1024, 33, 16), (2048, 100, 16)])
def test_resident_vs_numpy(gol, N, gens, kin):
    s = _sim(gol, N, kernel_depth=kin).init(5, seed=N + gens)
    s.step(gens)
    st = s.stats()
    assert st["kernel"].startswith(f"resident@{kin}"), st
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, N + gens), gens))


def test_resident_repeated_runs_and_graphs(gol):
    """Consecutive run() calls (per-tile superstep counters carry over launches), the hinted run as a
    replayed graph, and lengths that are not multiples of the halo depth."""
    N = 512
    s = _sim(gol, N, run_hint=50).init(5, seed=7)
    ref = initial_board(5, N, 1, True, 7)
    for g in (50, 50, 13, 1, 50, 96):
        s.step(g)
        ref = numpy_step(ref, g)
        assert np.array_equal(s.board(), ref), g
    assert s.stats()["graph_launches"] >= 3


def test_resident_rectangular(gol):
    N, W, gens = 300, 1024, 45
    s = _sim(gol, N, width=W, kernel_depth=12).init(5, seed=3)
    s.step(gens)
    from gol_amd.ops import random_board

    ref = numpy_step(random_board(N, W, 3), gens)
    assert np.array_equal(s.board(), ref)


def test_resident_config2_vs_torch(gol):
    import torch

    N, seed = 8192, 0x5EED
    s = _sim(gol, N, run_hint=1000).init(5, seed=seed)
    ref = torch.as_tensor(initial_board(5, N, 1, True, seed), device="cuda:0")
    for g in (100, 37):
        s.step(g)
        ref = torch_step(ref, g, device="cuda:0")
        got = s.board()
        assert np.array_equal(got, ref.cpu().numpy()), f"{int((got != ref.cpu().numpy()).sum())} cells differ"
    assert s.population() == int(ref.sum(dtype=torch.int64).item())


def test_resident_refuses_unfit_boards(gol):
    with pytest.raises(Exception, match="resident"):
        _sim(gol, 100).init(5, seed=1)  # width % 64 != 0


def test_resident_timeout_drops_candidate(gol, monkeypatch):
    """A resident candidate whose neighbour waits time out in the init timing (GOL_RESIDENT_TIMEOUT_TICKS=0:
    the first unsatisfied wait gives up) is dropped by the auto kernel choice, the board stays exact,
    and only a forced GOL_KERNEL=resident fails."""
    monkeypatch.setenv("GOL_RESIDENT_TIMEOUT_TICKS", "0")
    N = 1024
    s = _sim(gol, N, kernel="auto", subtiles=0).init(5, seed=11)
    assert not s.stats()["kernel"].startswith("resident"), s.stats()
    s.step(40)
    assert np.array_equal(s.board(), numpy_step(initial_board(5, N, 1, True, 11), 40))
    with pytest.raises(Exception, match="timed out"):
        _sim(gol, N, kernel="resident").init(5, seed=11)

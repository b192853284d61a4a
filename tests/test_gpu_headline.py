"""The exact headline configuration (bench.py, BASELINE.json metric) against an independent oracle.

32768^2 board, every setting at its default (auto): halo depth 128, the schedule the init-time
measurement picks (two sub-tiles on two streams, or one tile), measured pass cuts, the run-length
hint of the driver's bench (20 timed generations after 5 warmup ones).  The full board is compared
with a PyTorch fp32 conv2d torus step on cuda:0 (exact for neighbour counts <= 8) after the driver's
cut (5 + 20 generations) and after 150 generations.  Rule: gol-with-cuda.cu:239-257.
"""
import numpy as np
import pytest

from gol_amd.ops import initial_board, torch_step

pytestmark = pytest.mark.gpu


def test_headline_32768_default_path(gol):
    import torch

    N, seed = 32768, 0x5EED
    sim = gol.Simulation(N, backend="hip", device=0, run_hint=20).init(5, seed=seed)
    st = sim.stats()
    assert st["depth"] == 128, st
    assert st["schedule"] in ("local", "local+subtiles2"), st
    ref = torch.as_tensor(initial_board(5, N, 1, True, seed), device="cuda:0")
    sim.step(5)
    sim.step(20)
    ref = torch_step(ref, 25, device="cuda:0")
    got = sim.board()
    assert np.array_equal(got, ref.cpu().numpy()), f"{int((got != ref.cpu().numpy()).sum())} cells differ"
    sim.step(125)
    ref = torch_step(ref, 125, device="cuda:0")
    got = sim.board()
    assert np.array_equal(got, ref.cpu().numpy()), f"{int((got != ref.cpu().numpy()).sum())} cells differ"
    assert sim.population() == int(ref.sum(dtype=torch.int64).item())


@pytest.mark.parametrize("N,decomp,hint", [(16384, "1d", 20), (16384, "2d", 400)])
def test_one_tile_auto_kernel_bench_cut(gol, N, decomp, hint):
    """One tile without neighbours, every setting auto, no sub-tiles (the tile kernel is too big for this
    board, so the autotune's full-tile kernel is step_temporal or step_pipe and its passes may sit at
    step_pipe depths): init (kernel autotune, pass costs with step_pipe geometries, the end-of-init
    prediction on a board snapshot) and the bench cut stay exact against the PyTorch oracle.  (A round-5
    tree built interior / band plans of split supersteps for such boards and failed at init on BASELINE
    config 4's 65536^2 board, 2-D.)"""
    import torch

    seed = 0x5EED
    sim = gol.Simulation(N, backend="hip", device=0, run_hint=hint, decomp=decomp, subtiles=0).init(5, seed=seed)
    st = sim.stats()
    assert st["predicted_us_per_gen"] > 0, st
    ref = torch.as_tensor(initial_board(5, N, 1, True, seed), device="cuda:0")
    sim.step(5)
    sim.step(hint)
    ref = torch_step(ref, 5 + hint, device="cuda:0")
    got = sim.board()
    assert np.array_equal(got, ref.cpu().numpy()), f"{int((got != ref.cpu().numpy()).sum())} cells differ"

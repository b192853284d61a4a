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

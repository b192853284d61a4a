"""full+gate at P = 8 thread ranks sharing one GPU (p2p emulation of RCCL's data plane), the driver's 5 + 20
cut, exact against the numpy torus oracle.

The gate needs each rank's compute and comm streams on hardware queues of their own (a flag write queued
behind its own gated kernel on a shared queue would wait for it): 8 ranks x 2 streams do not fit the default
GPU_MAX_HW_QUEUES = 4, so the ranks run in a child process with GPU_MAX_HW_QUEUES = 32 and GOL_GATE = 1 (the
gate is otherwise only eligible with an RCCL transport, one rank per GPU).  Reference loop: gol-main.c:84-116.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, threading
import numpy as np
sys.path.insert(0, sys.argv[1])
import gol_amd as gol
from gol_amd.ops import numpy_step, random_board
P, H, W, SEED = 8, 1024, 2048, 41
ts = gol.parallel.p2p_thread_transports(P)
out, errs = [None] * P, []
def rank_main(r):
    try:
        s = gol.Simulation(P * H, ts[r], backend="hip", device=0, global_mode=True, width=W, halo_depth=32,
                           run_hint=20, schedule="gate", subtiles=0, kernel="temporal")
        s.init(5, seed=SEED)
        st = s.stats()
        assert st["schedule"] == "full+gate", st
        s.step(5)
        s.step(20)
        out[r] = (s.geometry.row0, s.board(), s.stats())
    except Exception as e:
        errs.append(f"rank {r}: {e!r}")
th = [threading.Thread(target=rank_main, args=(r,)) for r in range(P)]
for t in th: t.start()
for t in th: t.join(timeout=200)
assert not errs, errs
board = np.zeros((P * H, W), dtype=np.uint8)
for r0, b, st in out:
    assert st["exchanges"] >= 2 and st["generations"] == 25, st
    board[r0:r0 + H] = b
want = numpy_step(random_board(P * H, W, SEED), 25)
assert np.array_equal(board, want), f"{int((board != want).sum())} cells differ"
print("p8 gate exact")
"""


def test_p8_gate_bench_cut(gol):
    env = dict(os.environ, GPU_MAX_HW_QUEUES="32", GOL_GATE="1", GOL_GRAPH_RCCL="0", GOL_SPINUP_MS="0")
    r = subprocess.run([sys.executable, "-c", CHILD, REPO], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "p8 gate exact" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])

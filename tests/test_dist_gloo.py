"""Multi-process torch.distributed (gloo, CPU): the engine's control and data planes over
``gol_amd.parallel.torch_transport`` — the same process model the GPU runs use with RCCL."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r"""
import os, sys, json
sys.path.insert(0, {repo!r})
import numpy as np
import gol_amd
from gol_amd.parallel import init_distributed, torch_transport
rank, P, local, grp = init_distributed(backend="gloo")
t = torch_transport(grp)
kw = json.loads(os.environ["GOL_TEST_KW"])
s = gol_amd.Simulation(int(os.environ["GOL_TEST_N"]), t, backend="cpu", **kw).init(5, seed=17)
s.step(int(os.environ["GOL_TEST_G"]))
np.save(os.path.join(os.environ["GOL_TEST_OUT"], f"r{{rank}}.npy"), s.board())
fp = s.fingerprint()
s.dump(os.path.join(os.environ["GOL_TEST_OUT"], f"Rank_{{rank}}_of_{{P}}.txt"))
print(json.dumps({{"rank": rank, "row0": s.geometry.row0, "col0": s.geometry.col0, "fp": fp}}))
import torch.distributed as dist
dist.destroy_process_group()
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("P,kw", [(2, {}), (2, {"decomp": "2d", "grid": "2x1", "global_mode": True, "halo_depth": 5}),
                                  (4, {"decomp": "2d", "grid": "2x2", "global_mode": True}),
                                  (6, {"decomp": "2d", "grid": "3x2", "global_mode": True})])
def test_gloo_multiprocess(tmp_path, P, kw):
    import json

    N, gens = 256, 17
    script = tmp_path / "w.py"
    script.write_text(WORKER.format(repo=REPO))
    port = _free_port()
    procs = []
    for r in range(P):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(P), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), GOL_TEST_N=str(N), GOL_TEST_G=str(gens), GOL_TEST_OUT=str(tmp_path),
                   GOL_TEST_KW=json.dumps(kw), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=240) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-2000:] for o in outs]
    infos = [json.loads(o[0].strip().splitlines()[-1]) for o in outs]
    from gol_amd.ops import initial_board, numpy_step

    per_rank = not kw.get("global_mode", False)
    ref = numpy_step(initial_board(5, N, P, per_rank, 17), gens)
    full = np.zeros_like(ref)
    for info in infos:
        b = np.load(tmp_path / f"r{info['rank']}.npy")
        full[info["row0"] : info["row0"] + b.shape[0], info["col0"] : info["col0"] + b.shape[1]] = b
    assert np.array_equal(full, ref)
    assert len({i["fp"] for i in infos}) == 1
    # the reference-format dumps (2-D: tile/strip blocks routed point to point over gloo)
    from gol_amd.utils import read_dump

    parts = sorted(read_dump(str(tmp_path / f"Rank_{r}_of_{P}.txt"))[1:] for r in range(P))
    assert np.array_equal(np.vstack([c for _, c in parts]), ref)

"""gol-mi355x: an MI355X-native (gfx950 / CDNA4) Conway's Game of Life stencil engine.

Capabilities of shoron-dutta/Game-of-Life---MPI-CUDA, re-designed for MI355X:

* native C++/HIP core (``_gol``): bit-packed boards, a hand-written temporal-blocked gfx950 kernel
  (v_bitop3 / v_alignbit / DPP), RCCL halo exchange over xGMI with comm/compute overlap and
  hipGraph-captured supersteps, 1-D row-strip and 2-D block decomposition, CPU backend;
* the reference CLI contract (``gol`` binary, ``python -m gol_amd``), dump format and patterns;
* Python API: :class:`gol_amd.models.Simulation`, oracles in :mod:`gol_amd.ops`, torch.distributed
  integration in :mod:`gol_amd.parallel`, dump/metrics helpers in :mod:`gol_amd.utils`.
"""
from ._native import _gol as native  # noqa: F401

__version__ = "0.1.0"

from .models import Simulation  # noqa: E402,F401
from . import models, ops, parallel, utils  # noqa: E402,F401

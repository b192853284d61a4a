"""The flagship "model": a Game of Life simulation on one rank of a (possibly multi-GPU) job.

Reference behaviour being reproduced (cited for parity checks):

* board = P stacked N x N tiles forming a (P*N) x N torus (``gol-main.c:76``, ``gol-main.c:84-87``);
* rule B3/S23 (``gol-with-cuda.cu:239-257``);
* patterns 0-4 (``gol-with-cuda.cu:55-171``) plus pattern 5 (seeded random, decomposition-invariant);
* per-rank dump files (``gol-main.c:17-28, 64-73, 134-139``).

The heavy lifting is native: :class:`Simulation` drives a ``_gol.Engine`` (HIP or CPU backend).
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np

from .._native import _gol
from ..ops.bitpack import unpack_words


def _tri(name: str) -> int:
    """GOL_* switch with an auto default: 1 on, 0 off, -1 auto (the engine decides by measurement)."""
    v = os.environ.get(name, "auto")
    return -1 if v == "auto" else int(int(v) != 0)


def default_backend() -> str:
    b = os.environ.get("GOL_BACKEND", "auto")
    if b != "auto":
        return b
    return "hip" if _gol.hip_device_count() > 0 else "cpu"


class Simulation:
    """One rank's view of a Game of Life job.

    Parameters
    ----------
    N:            the reference ``worldSize`` (per-rank tile side), or the global side with ``global_mode``.
    transport:    a ``_gol.Transport``; defaults to a single-rank transport.  See
                  :mod:`gol_amd.parallel` for torch.distributed / RCCL / thread transports.
    backend:      ``"hip"``, ``"cpu"`` or ``"auto"``.
    halo_depth:   generations per halo exchange (<= 128 in 1-D, <= 63 in 2-D; 0 = auto, as in
                  Engine::Engine: 128 for 1-D strips of >= 2048 rows with neighbours (or the
                  self-exchange) and for ranks that can run two sub-tiles, 56 for 2-D tiles of >= 2048
                  rows with neighbours, otherwise 32).  The rule is B3/S23 (Conway), the only rule
                  the bit-sliced kernels implement.
    kernel_depth: generations per kernel pass (HIP; 0 = auto).  A superstep of halo_depth
                  generations runs as several kernel passes in 1-D (communication-avoiding halos).
    kernel:       HIP stencil kernel: ``"auto"`` (candidates timed at init), ``"temporal"``,
                  ``"tile"``, ``"pipe"`` (level-pipelined workgroups; geometry GOL_PIPE=nw,L,wg),
                  ``"resident"`` or ``"lds"`` (GOL_KERNEL).
    decomp/grid:  ``"1d"`` row strips (reference) or ``"2d"`` blocks, optional ``"PxxPy"`` grid.
    width:        board columns (0 = N: the reference's square tiles).  With ``width`` the per-rank
                  strip (or, in global mode, the board) is N rows x ``width`` columns.
    compat:       reproduce the reference's halo quirks (frozen gen-0 halos, P<=2 swap).
    watchdog:     seconds without progress before the job is aborted (0 = off; GOL_WATCHDOG).
    """

    def __init__(
        self,
        N: int,
        transport=None,
        *,
        backend: str = "auto",
        global_mode: bool = False,
        decomp: str = "1d",
        grid: str = "",
        halo_depth: int = int(os.environ.get("GOL_HALO_DEPTH", "0")),
        kernel_depth: int = int(os.environ.get("GOL_KERNEL_DEPTH", "0")),
        overlap: bool = True,
        graph: bool = True,
        compat: bool = False,
        device: Optional[int] = None,
        kernel: str = os.environ.get("GOL_KERNEL", "auto"),
        rows_per_wave: int = 0,
        waves_target: int = 0,
        profile: bool = False,
        watchdog: float = float(os.environ.get("GOL_WATCHDOG", "0")),
        tile_waves: int = int(os.environ.get("GOL_TILE_WAVES", "8")),
        force_split: bool = os.environ.get("GOL_FORCE_SPLIT", "0") == "1",
        schedule: str = os.environ.get("GOL_SCHEDULE", "auto"),
        run_hint: int = 0,
        sub_occ: int = int(os.environ.get("GOL_SUB_OCC", "2")),
        self_exchange: bool = os.environ.get("GOL_SELF_EXCHANGE", "0") == "1",
        subtiles: int = -1 if os.environ.get("GOL_SUBTILES", "auto") == "auto" else int(os.environ["GOL_SUBTILES"]),
        width: int = 0,
        subtile_overlap: Optional[int] = None,
    ):
        self.transport = transport if transport is not None else _gol.SelfTransport()
        P, rank = self.transport.size(), self.transport.rank()
        self.backend = default_backend() if backend == "auto" else backend
        self.decomposition = _gol.make_decomposition(N, P, global_mode, decomp, grid, int(width))
        self.geometry = _gol.make_geometry(self.decomposition, rank)
        cfg = _gol.EngineConfig()
        cfg.backend = self.backend
        cfg.halo_depth = halo_depth
        cfg.kernel_depth = kernel_depth
        cfg.overlap = overlap
        cfg.graph = graph
        cfg.compat = compat
        cfg.kernel = kernel
        cfg.subtiles = int(subtiles)  # 2 / 0 / -1 auto: two sub-tiles per rank on two streams (HIP, 1-D)
        cfg.run_hint = int(run_hint)  # generations of the runs to come: one replay graph covers them
        cfg.rows_per_wave = rows_per_wave
        cfg.waves_target = waves_target
        cfg.profile = profile
        cfg.watchdog_s = float(watchdog)
        cfg.tile_waves = int(tile_waves)
        cfg.tune_tile_waves = "GOL_TILE_WAVES" not in os.environ
        cfg.sub_occ = int(sub_occ)
        # 1 on / 0 off / -1 auto: a candidate of the init-time schedule timing (GOL_* env defaults)
        if subtile_overlap is None:  # 0 off, 1 on (half 0's interior overlaps the exchange), auto: timed
            v = os.environ.get("GOL_SUBTILE_OVERLAP", "auto")
            subtile_overlap = -1 if v == "auto" else int(v)
        cfg.subtile_overlap = int(subtile_overlap)
        cfg.self_exchange = bool(self_exchange)
        cfg.force_split = bool(force_split)
        cfg.sched = schedule
        cfg.graph_rccl = _tri("GOL_GRAPH_RCCL")
        cfg.plan_xcds = int(os.environ.get("GOL_PLAN_XCDS", "8"))
        if self.backend == "hip":
            n = _gol.hip_device_count()
            if n <= 0:
                raise RuntimeError("backend 'hip' requested but no HIP device is visible")
            cfg.device = (rank if device is None else device) % n
        self.config = cfg
        self.engine = _gol.Engine.create(self.geometry, cfg, self.transport)
        self.pattern = None

    # -- lifecycle -------------------------------------------------------------------------
    def init(self, pattern: int = 5, seed: int = 0x5EED) -> "Simulation":
        self.pattern = _gol.make_pattern(pattern, self.decomposition, seed)
        self.engine.init(self.pattern)
        return self

    def step(self, generations: int = 1) -> "Simulation":
        self.engine.run(int(generations))
        return self

    run = step

    def synchronize(self) -> None:
        self.engine.synchronize()

    # -- state -----------------------------------------------------------------------------
    @property
    def generation(self) -> int:
        return self.engine.generation

    def words(self) -> np.ndarray:
        """Local tile as packed uint64 words, shape (h, ceil(w/64)); bit b of word c = column 64c+b."""
        return self.engine.tile_words()

    def board(self) -> np.ndarray:
        """Local tile as a (h, w) uint8 array of 0/1 cells."""
        return unpack_words(self.words(), self.geometry.w)

    def set_board(self, cells: np.ndarray) -> None:
        from ..ops.bitpack import pack_cells

        cells = np.asarray(cells)
        if cells.shape != (self.geometry.h, self.geometry.w):
            raise ValueError(f"expected a {(self.geometry.h, self.geometry.w)} board, got {cells.shape}")
        self.engine.set_tile_words(pack_cells(cells))

    def population(self) -> int:
        """Global live-cell count (collective)."""
        return int(self.engine.population())

    def fingerprint(self) -> int:
        """Decomposition-invariant fingerprint of the global board (collective)."""
        return int(self.engine.fingerprint())

    def stats(self) -> dict:
        return self.engine.stats()

    def describe(self) -> str:
        return self.engine.describe()

    # -- I/O -------------------------------------------------------------------------------
    def dump(self, path: Optional[str] = None) -> str:
        """Write this rank's reference-format dump file (collective); returns the path."""
        if path is None:
            path = _gol.dump_filename(self.geometry.rank, self.decomposition.P)
        _gol.write_dumps(self.engine, path)
        return path

    def checkpoint(self, prefix: str) -> None:
        """Write ``<prefix>.gol`` (collective): the global board, each rank writing its own rectangle.

        The file does not depend on the decomposition: :meth:`restore` works on any rank count or
        grid with the same global board size.
        """
        _gol.save_checkpoint(self.engine, prefix, self.pattern.seed if self.pattern else 0)

    def restore(self, prefix: str) -> int:
        """Load this rank's rectangle of ``<prefix>.gol``; returns the snapshot's generation."""
        return int(_gol.load_checkpoint(self.engine, prefix))

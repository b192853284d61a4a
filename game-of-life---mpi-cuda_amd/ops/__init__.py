"""Ops: bit packing, oracles (numpy / torch conv2d / reference-quirk model) and direct access to the
native kernels through the ``_gol`` extension."""
from .bitpack import pack_cells, unpack_words  # noqa: F401
from .oracle import initial_board, numpy_step, quirk_model, random_board, torch_step  # noqa: F401
from .._native import _gol as _native


def cpu_torus_step(words, width: int, generations: int = 1):
    """Native CPU stepper (bit-sliced) on dense packed words (h, nw) of a full torus."""
    return _native.cpu_torus_step(words, width, generations)


def naive_byte_run(N: int, generations: int, threads: int = 256, sync_each: bool = True, seed: int = 0x5EED):
    """Reference-class GPU yardstick (byte per cell, thread per cell). Returns (seconds, population)."""
    return _native.naive_byte_run(N, generations, threads, sync_each, seed)


def build_plan(regions, nw, h, rows_per_chunk, k, xwrap=False, fold=False):
    """Lane descriptors of the temporal kernel's work plan: (array[n_lanes, 4], stats).

    fold=True: the folded tile kernel's plan (32-lane tiles, lanes 32-63 repeat lanes 0-31)."""
    return _native.build_plan(regions, nw, h, rows_per_chunk, k, xwrap, fold)

"""Bit packing helpers (numpy): 64 cells per uint64 word, bit b of word c = column 64*c + b.

Matches the native tile layout (csrc/include/gol/geometry.hpp) so Python oracles and the engine
exchange boards without conversion errors.  Relies on a little-endian host (x86-64).
"""
import numpy as np


def pack_cells(cells: np.ndarray) -> np.ndarray:
    """(h, w) 0/1 array -> (h, ceil(w/64)) uint64 words (bits beyond w are zero)."""
    cells = np.asarray(cells).astype(np.uint8) & 1
    h, w = cells.shape
    nw = (w + 63) // 64
    padded = np.zeros((h, nw * 64), dtype=np.uint8)
    padded[:, :w] = cells
    return np.ascontiguousarray(np.packbits(padded, axis=1, bitorder="little")).view(np.uint64).reshape(h, nw)


def unpack_words(words: np.ndarray, w: int) -> np.ndarray:
    """(h, nw) uint64 words -> (h, w) uint8 cells."""
    words = np.ascontiguousarray(words, dtype=np.uint64)
    h, nw = words.shape
    b = words.view(np.uint8).reshape(h, nw * 8)
    return np.unpackbits(b, axis=1, bitorder="little")[:, :w].copy()

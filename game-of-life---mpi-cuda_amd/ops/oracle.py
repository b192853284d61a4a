"""Independent oracles for testing the native engine.

* :func:`numpy_step` — byte-per-cell torus step (numpy roll), the plain reference.
* :func:`torch_step` — the same with a 3x3 ``conv2d`` and circular padding in fp32; runs on the GPU
  (PyTorch-ROCm) to cross-check large boards independently of the HIP kernels.
* :func:`quirk_model` — the reference's actual behaviour (survey Q1-Q3): every rank steps its tile
  with x-wrap and CONSTANT ghost rows taken from the generation-0 boards, with the P <= 2 swap.
* :func:`initial_board` — pattern placement mirror (patterns 0-5) computed in Python, including the
  splitmix64-based random pattern, to check the native init bit-for-bit.
"""
from __future__ import annotations

import numpy as np

MASK64 = (1 << 64) - 1


def numpy_step(board: np.ndarray, generations: int = 1) -> np.ndarray:
    b = np.asarray(board, dtype=np.uint8)
    for _ in range(generations):
        n = sum(
            np.roll(np.roll(b, dy, axis=0), dx, axis=1)
            for dy in (-1, 0, 1)
            for dx in (-1, 0, 1)
            if dy or dx
        )
        b = ((n == 3) | ((b == 1) & (n == 2))).astype(np.uint8)
    return b


def torch_step(board, generations: int = 1, device=None):
    """B3/S23 on a torus with torch conv2d (fp32, exact for counts <= 8).  Returns a torch uint8 tensor."""
    import torch
    import torch.nn.functional as F

    if isinstance(board, torch.Tensor):  # e.g. a previous torch_step result, already on the device
        x = board.to(device=device if device is not None else board.device, dtype=torch.float32)[None, None]
    else:
        x = torch.as_tensor(np.asarray(board), dtype=torch.float32, device=device)[None, None]
    k = torch.ones(1, 1, 3, 3, dtype=torch.float32, device=x.device)
    k[0, 0, 1, 1] = 0
    for _ in range(generations):
        n = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="circular"), k)
        x = ((n == 3) | ((x == 1) & (n == 2))).to(torch.float32)
    return x[0, 0].to(torch.uint8)


def _mix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def random_word(seed: int, grow: int, gword: int, gwords: int) -> int:
    return _mix64(((seed * 0xD1B54A32D192ED03) & MASK64) ^ _mix64((grow * gwords + gword) & MASK64))


def _mix64_np(z: np.ndarray) -> np.ndarray:
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def random_board(H: int, W: int, seed: int) -> np.ndarray:
    """Pattern 5 on an H x W global board, vectorised (identical to the native counter hash)."""
    gw = (W + 63) // 64
    with np.errstate(over="ignore"):
        r = np.arange(H, dtype=np.uint64)[:, None]
        c = np.arange(gw, dtype=np.uint64)[None, :]
        idx = r * np.uint64(gw) + c
        sm = np.uint64((seed * 0xD1B54A32D192ED03) & MASK64)
        words = _mix64_np(sm ^ _mix64_np(idx))
    from .bitpack import unpack_words

    return unpack_words(words, W)


def strips(H: int, N: int, P: int, per_rank: bool):
    if per_rank:
        return [(s * N, (s + 1) * N) for s in range(P)]
    base, extra = divmod(H, P)
    out, pos = [], 0
    for s in range(P):
        n = base + (1 if s < extra else 0)
        out.append((pos, pos + n))
        pos += n
    return out


def initial_board(pattern: int, N: int, P: int = 1, per_rank: bool = True, seed: int = 0x5EED) -> np.ndarray:
    """Global initial board for the reference patterns (gol-with-cuda.cu:55-171) + pattern 5."""
    H = N * P if per_rank else N
    W = N
    b = np.zeros((H, W), dtype=np.uint8)
    st = strips(H, N, P, per_rank)

    def flat(s, f):
        r0, r1 = st[s]
        hs = r1 - r0
        if 0 <= f < hs * W:
            b[r0 + f // W, f % W] = 1

    if pattern == 0:
        pass
    elif pattern == 1:
        b[:] = 1
    elif pattern == 2:
        for s, (r0, r1) in enumerate(st):
            hs = r1 - r0
            off = (hs - 1) * W
            for j in range(127, 137):
                if off + j < hs * W:
                    flat(s, off + j)
    elif pattern == 3:
        flat(0, 0)
        flat(0, W - 1)
        if P > 1:
            hs = st[-1][1] - st[-1][0]
            flat(P - 1, (hs - 1) * W)
            flat(P - 1, (hs - 1) * W + W - 1)
    elif pattern == 4:
        flat(0, 0)
        flat(0, 1)
        flat(0, W - 1)
    elif pattern == 5:
        b = random_board(H, W, seed)
    else:
        raise ValueError(f"Pattern {pattern} has not been implemented")
    return b


def _step_with_ghosts(tile: np.ndarray, above: np.ndarray, below: np.ndarray) -> np.ndarray:
    ext = np.vstack([above[None, :], tile, below[None, :]]).astype(np.uint8)
    n = sum(
        np.roll(ext, dx, axis=1)[1 + dy : 1 + dy + tile.shape[0]]
        for dy in (-1, 0, 1)
        for dx in (-1, 0, 1)
        if dy or dx
    )
    return ((n == 3) | ((tile == 1) & (n == 2))).astype(np.uint8)


def quirk_model(init: np.ndarray, P: int, generations: int) -> np.ndarray:
    """Reference behaviour (GOL_COMPAT=reference): frozen gen-0 halos, swapped for P <= 2."""
    H, W = init.shape
    N = H // P
    tiles = [init[r * N : (r + 1) * N].copy() for r in range(P)]
    above, below = [], []
    for r in range(P):
        prev, nxt = tiles[(r - 1) % P], tiles[(r + 1) % P]
        if P >= 3:
            above.append(prev[-1].copy())
            below.append(nxt[0].copy())
        else:
            above.append(prev[0].copy())
            below.append(nxt[-1].copy())
    for _ in range(generations):
        tiles = [_step_with_ghosts(tiles[r], above[r], below[r]) for r in range(P)]
    return np.vstack(tiles)

"""Parallelism: spatial domain decomposition (1-D row strips / 2-D blocks with corner halos) across
ranks, one process per GPU, RCCL halo exchange over xGMI (see :mod:`.dist`)."""
from .dist import (  # noqa: F401
    env_rank,
    init_distributed,
    p2p_thread_transports,
    rccl_transport,
    tcp_transport,
    thread_transports,
    torch_transport,
)
from .._native import _gol as _native


def decomposition(N: int, P: int, global_mode: bool = False, decomp: str = "1d", grid: str = "", width: int = 0):
    """The native decomposition (tile extents per rank, process grid, dump strips); width 0 = square."""
    return _native.make_decomposition(N, P, global_mode, decomp, grid, width)

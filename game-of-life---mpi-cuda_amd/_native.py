"""Loader for the native extension ``_gol`` (built in-tree by ``__graft_entry__.build()``).

``torch`` is imported first when available so the extension binds to the HIP runtime torch already
loaded (same SONAME ``libamdhip64.so.7``) instead of loading a second copy.  A missing extension is a
hard error: there is no pure-Python fallback for the compute path.
"""
import importlib
import os
import sys

try:  # share torch's HIP runtime / RCCL when both are used in one process
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the native core
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))


def load():
    if _HERE not in sys.path:
        sys.path.insert(0, _HERE)
    try:
        return importlib.import_module("_gol")
    except ImportError as e:  # pragma: no cover
        raise ImportError(
            "gol native extension _gol is not built; run `python -c 'import __graft_entry__ as g; g.build()'` "
            f"(or cmake -S . -B build -G Ninja && cmake --build build) first: {e}"
        ) from e


_gol = load()

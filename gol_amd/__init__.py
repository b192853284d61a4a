"""Import alias for the ``game-of-life---mpi-cuda_amd`` package directory.

The package lives in a directory whose name is not a Python identifier; this shim makes it
importable as ``gol_amd`` (``import gol_amd``, ``from gol_amd.models import Simulation``) by pointing
the package search path at that directory and executing its ``__init__``.
"""
import os as _os

_real = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "game-of-life---mpi-cuda_amd")
__path__ = [_real]
__file__ = _os.path.join(_real, "__init__.py")
with open(__file__) as _f:
    exec(compile(_f.read(), __file__, "exec"))

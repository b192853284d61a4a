"""Models: the Game of Life simulation (B3/S23) driven by the native engine."""
from .life import Simulation, default_backend  # noqa: F401

"""Utilities: native build driver, dump-file reader/writer, CLI entry, metrics."""
from .dumpfile import format_dump, header, read_dump  # noqa: F401


def run_cli(args):
    """Run the reference-compatible CLI in-process (``args`` excludes the program name)."""
    from .._native import _gol

    return _gol.run_cli(["gol", *map(str, args)])

"""Reader/writer for the reference board-dump format (``Rank_<r>_of_<P>.txt``).

Format (gol-main.c:17-28, 136):
    ######################### FINAL WORLD IN RANK <r> IS ###############################
    Row %2d: c c c ... c \n         (one line per row; each cell "%u " incl. trailing space)
The reference has no reader; this one exists for tests and tooling.
"""
from __future__ import annotations

import re

import numpy as np

HEADER_RE = re.compile(r"^#{25} FINAL WORLD IN RANK (\d+) IS #{31}$")


def header(rank: int) -> str:
    return "#" * 25 + f" FINAL WORLD IN RANK {rank} IS " + "#" * 31 + "\n"


def format_dump(rank: int, cells: np.ndarray, first_row: int) -> str:
    lines = [header(rank)]
    for i, row in enumerate(np.asarray(cells, dtype=np.uint8)):
        lines.append("Row %2d: " % (first_row + i) + "".join("%u " % v for v in row) + "\n")
    return "".join(lines)


def read_dump(path: str):
    """Returns (rank, first_row, cells[h, w])."""
    with open(path) as f:
        text = f.read()
    lines = text.split("\n")
    m = HEADER_RE.match(lines[0])
    if not m:
        raise ValueError(f"{path}: bad header {lines[0]!r}")
    rows, first = [], None
    for ln in lines[1:]:
        if not ln:
            continue
        label, _, rest = ln.partition(": ")
        if first is None:
            first = int(label.split()[1])
        rows.append([int(t) for t in rest.split()])
    cells = np.array(rows, dtype=np.uint8) if rows else np.zeros((0, 0), np.uint8)
    return int(m.group(1)), (first or 0), cells

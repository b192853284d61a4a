"""Runs the C++ unit-test binary (host-only: CLI parsing, geometry, patterns, planner, CPU stepper,
dump formatting, multi-rank thread engines, compat mode)."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gol_unit():
    r = subprocess.run([os.path.join(REPO, "build", "gol_unit")], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert ", 0 failed" in r.stdout

"""Native build driver: configure + build the CMake project (gfx950) in-tree.

Produces ``build/gol`` (CLI), ``build/gol_unit`` (C++ tests) and the Python extension
``game-of-life---mpi-cuda_amd/_gol*.so``.  Used by ``__graft_entry__.build()`` and the test suite.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BUILD = os.path.join(REPO, "build")
PKG = os.path.join(REPO, "game-of-life---mpi-cuda_amd")


def _env():
    env = dict(os.environ)
    rocm = "/opt/rocm"
    env["PATH"] = f"{rocm}/bin:{rocm}/lib/llvm/bin:" + env.get("PATH", "")
    env.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
    return env


def build(jobs: int | None = None, verbose: bool = False, build_type: str = "Release") -> None:
    jobs = jobs or min(16, os.cpu_count() or 8)
    env = _env()
    generator = ["-G", "Ninja"] if shutil.which("ninja") or os.path.exists("/usr/bin/ninja") else []
    cfg = [
        "cmake", "-S", REPO, "-B", BUILD, *generator,
        f"-DCMAKE_BUILD_TYPE={build_type}",
        "-DCMAKE_PREFIX_PATH=/opt/rocm",
        "-DCMAKE_HIP_COMPILER=/opt/rocm/lib/llvm/bin/clang++",
        "-DCMAKE_HIP_ARCHITECTURES=gfx950",
        f"-DPython3_EXECUTABLE={sys.executable}",
    ]
    out = None if verbose else subprocess.DEVNULL
    if not os.path.exists(os.path.join(BUILD, "CMakeCache.txt")):
        subprocess.run(cfg, check=True, env=env, stdout=out)
    r = subprocess.run(["cmake", "--build", BUILD, "-j", str(jobs)], env=env, capture_output=True, text=True)
    if r.returncode != 0:
        # a stale cache (moved checkout / new toolchain): reconfigure once
        subprocess.run(cfg, check=True, env=env, stdout=out)
        r = subprocess.run(["cmake", "--build", BUILD, "-j", str(jobs)], env=env, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout[-20000:] + r.stderr[-20000:])
        raise RuntimeError("native build failed")
    if not glob.glob(os.path.join(PKG, "_gol*.so")):
        raise RuntimeError("native build did not produce the _gol extension")


def gol_binary() -> str:
    return os.path.join(BUILD, "gol")


def ensure_built() -> None:
    if not (glob.glob(os.path.join(PKG, "_gol*.so")) and os.path.exists(gol_binary())):
        build()

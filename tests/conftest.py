import glob
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer multi-process tests")


def _ensure_native():
    pkg = os.path.join(REPO, "game-of-life---mpi-cuda_amd")
    if not glob.glob(os.path.join(pkg, "_gol*.so")) or not os.path.exists(os.path.join(REPO, "build", "gol")):
        import importlib.util

        spec = importlib.util.spec_from_file_location("_gol_build", os.path.join(pkg, "utils", "build.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        mod.build()


_ensure_native()


@pytest.fixture(scope="session")
def gol():
    import gol_amd

    return gol_amd


@pytest.fixture(scope="session")
def gol_bin():
    return os.path.join(REPO, "build", "gol")


@pytest.fixture(scope="session")
def has_gpu():
    import gol_amd

    return gol_amd.native.hip_device_count() > 0


def pytest_collection_modifyitems(config, items):
    import gol_amd

    if gol_amd.native.hip_device_count() > 0:
        return
    skip = pytest.mark.skip(reason="no HIP device")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)

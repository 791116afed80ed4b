import os
import sys

import pytest

# torch bundles its own HIP runtime: load it before libvio360.so so that both resolve to the same
# libamdhip64 (loaded the other way round, torch's lazy CUDA init finds no device)
try:
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def vio():
    import importlib
    return importlib.import_module("360_visual_inertial_odometry_amd")


@pytest.fixture(scope="session")
def synth():
    import importlib
    return importlib.import_module("360_visual_inertial_odometry_amd.synth")


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib
    return oracle_lib.load()


@pytest.fixture(scope="session")
def gpu_ctx(vio):
    ctx = vio.Context(0)
    yield ctx
    ctx.close()

"""Test configuration.

Markers: ``gpu`` — needs an MI355X (HIP device); the driver runs
``pytest -m "not gpu"`` on the CPU build box and ``pytest -m gpu`` on a GPU box.
GPU tests fail loudly if the native extension is missing (no silent
fallback); they skip only when no HIP device is visible at all.
"""

import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an MI355X GPU (HIP device)")
    config.addinivalue_line("markers", "slow: longer CPU tests")


@pytest.fixture(scope="session")
def pe():
    import poisson_ellipse_openmp_mpi_cuda_amd as pe

    pe.native()  # loud failure if the extension is not built
    return pe


@pytest.fixture(scope="session")
def nat(pe):
    return pe.native()


@pytest.fixture(scope="session")
def gpu(nat):
    if nat.device_count() < 1:
        pytest.skip("no HIP device visible")
    nat.set_device(0)
    return nat


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port

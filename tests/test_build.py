"""Build-system checks: the CMake project configures (the Makefile build is
exercised by every other test through the in-tree extension)."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cmake_configures(tmp_path):
    cmake = shutil.which("cmake")
    if cmake is None or not os.path.isdir("/opt/rocm"):
        pytest.skip("cmake / ROCm not available")
    gen = ["-G", "Ninja"] if shutil.which("ninja") else []
    r = subprocess.run([cmake, "-S", ROOT, "-B", str(tmp_path / "b"), *gen, "-DCMAKE_PREFIX_PATH=/opt/rocm"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert (tmp_path / "b" / ("build.ninja" if gen else "Makefile")).exists()

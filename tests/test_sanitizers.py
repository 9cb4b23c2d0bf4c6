"""Host sanitizer runs of the CPU solver (SURVEY §5 race detection): ASan +
UBSan over the serial and thread-rank × OpenMP paths, TSan over the thread-
rank transport.  GPU sanitizers are not available on the MI355X pool; device
races are covered by the bitwise-determinism tests in test_gpu.py."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def san_bins():
    if shutil.which("make") is None or shutil.which("g++") is None:
        pytest.skip("no host toolchain")
    r = subprocess.run(["make", "-s", "asan", "tsan"], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return os.path.join(ROOT, "bin", "pe_cpu_asan"), os.path.join(ROOT, "bin", "pe_cpu_tsan")


def _run(cmd, env=None):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=dict(os.environ, **(env or {})))
    return r.returncode, r.stdout + r.stderr


@pytest.mark.parametrize("args", [["--backend", "serial", "40", "40"],
                                  ["--backend", "ranks", "--ranks", "4", "--threads", "2", "100", "80"],
                                  ["--backend", "ranks", "--ranks", "3", "--decomp", "3x1", "60", "50"]])
def test_asan_ubsan_clean(san_bins, args):
    rc, out = _run([san_bins[0], *args], {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1"})
    assert rc == 0, out[-3000:]
    assert "AddressSanitizer" not in out and "runtime error" not in out
    assert "Iter=" in out


def test_tsan_thread_ranks_clean(san_bins):
    rc, out = _run([san_bins[1], "--backend", "ranks", "--ranks", "4", "--threads", "1", "100", "80"],
                   {"TSAN_OPTIONS": "halt_on_error=1"})
    assert rc == 0, out[-3000:]
    assert "ThreadSanitizer" not in out
    assert "Iter=102" in out

"""Output formats (reference stdout lines, JSON) and the CLI front ends."""

import json
import os
import subprocess
import sys

import numpy as np
import pytest

from poisson_ellipse_openmp_mpi_cuda_amd import EllipseProblem, solve
from poisson_ellipse_openmp_mpi_cuda_amd.utils import dump
from poisson_ellipse_openmp_mpi_cuda_amd.utils.report import json_report, legacy_lines, parse_legacy

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_legacy_lines_stage2_roundtrip():
    rep = solve(EllipseProblem(40, 40), backend="serial")
    text = legacy_lines(rep)
    assert "Converged after 50 iterations (||w(k+1)-w(k)|| < 1e-06)." in text
    p = parse_legacy(text)
    assert (p["M"], p["N"], p["iters"], p["converged"], p["tol"]) == (40, 40, 50, True, 1e-6)


def test_legacy_lines_stage4_labels():
    rep = solve(EllipseProblem(40, 40), backend="serial")
    rep.backend = "hip"
    text = legacy_lines(rep)
    for label in ("GPU compute time (Ap + D^{-1}r, max over ranks)", "Host<->Device copy time (max over ranks)",
                  "MPI halo exchange time (max over ranks)", "Preconditioner CPU part time (max over ranks)",
                  "Dot products time (max over ranks)", "Init time (program)", "Solver time (MPI+CUDA)",
                  "Finalization time"):
        assert label in text
    assert parse_legacy(text)["iters"] == 50


def test_json_report_schema():
    rep = solve(EllipseProblem(40, 40), backend="omp", threads=2)
    d = json.loads(json_report(rep, {"extra": 1}))
    for k in ("backend", "M", "N", "iters", "converged", "timers", "l2_err", "max_err", "iters_per_s", "Px", "Py"):
        assert k in d
    assert d["extra"] == 1 and d["iters"] == 50


def test_native_legacy_formatter(nat):
    rep = solve(EllipseProblem(40, 40), backend="serial")
    P = EllipseProblem(40, 40).to_native()
    res, _ = nat.cpu_solve(P, 1, nat.DecompMode.Reference, nat.SolveOptions(), False)
    text = nat.format_result_legacy(P, res, 1, "stage2")
    assert parse_legacy(text)["iters"] == rep.iters


def test_python_cli_serial(tmp_path):
    out = subprocess.run([sys.executable, "-m", "poisson_ellipse_openmp_mpi_cuda_amd", "--backend", "serial", "--json",
                          "--dump", str(tmp_path / "w.npy"), "--pgm", str(tmp_path / "w.pgm"), "40", "40"],
                         cwd=ROOT, capture_output=True, text=True, check=True).stdout
    assert parse_legacy(out)["iters"] == 50
    d = json.loads(out.strip().splitlines()[-1])
    assert d["iters"] == 50
    w, meta = dump.load(tmp_path / "w.npy")
    assert w.shape == (39, 39) and meta["iters"] == 50
    assert 0.09 < w.max() < 0.11  # peak ≈ u(0,0) = 0.1 (Этап3.pdf p.9)
    assert (tmp_path / "w.pgm").read_bytes().startswith(b"P5")


def test_native_cpu_app():
    exe = os.path.join(ROOT, "bin", "pe_cpu")
    if not os.path.exists(exe):
        pytest.skip("bin/pe_cpu not built")
    out = subprocess.run([exe, "--backend", "ranks", "--ranks", "4", "400", "600"], capture_output=True, text=True,
                         check=True).stdout
    assert "Pure MPI 2D run with 4 processes; M=400, N=600" in out
    assert parse_legacy(out)["iters"] == 546
    out = subprocess.run([exe, "--threads-sweep", "1,2", "--backend", "omp", "40", "40"], capture_output=True,
                         text=True, check=True).stdout
    assert out.count("Threads =") == 2


def test_native_stage0_grid_loop():
    """`pe_cpu --stage stage0` = the stage0 program (Withoutopenmp1.cpp:176-196):
    grids {10, 20, 40}², unweighted stop rule → 17 / 31 / 61 iterations."""
    import re

    exe = os.path.join(ROOT, "bin", "pe_cpu")
    if not os.path.exists(exe):
        pytest.skip("bin/pe_cpu not built")
    out = subprocess.run([exe, "--stage", "stage0"], capture_output=True, text=True, check=True).stdout
    got = [tuple(map(int, m)) for m in re.findall(r"M=(\d+), N=(\d+) \| Iter=(\d+) \| Time=\d+\.\d{4} s", out)]
    assert got == [(10, 10, 17), (20, 20, 31), (40, 40, 61)]


def test_dump_roundtrip(tmp_path):
    w = np.random.default_rng(0).random((5, 7))
    dump.save(tmp_path / "x.npy", w, EllipseProblem(6, 8))
    w2, meta = dump.load(tmp_path / "x.npy")
    assert np.array_equal(w, w2) and meta["M"] == 6

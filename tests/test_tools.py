"""Plot / summary tools run without a plotting library."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_plot_solution_and_scaling(tmp_path):
    from poisson_ellipse_openmp_mpi_cuda_amd import EllipseProblem, solve
    from poisson_ellipse_openmp_mpi_cuda_amd.utils import dump

    prob = EllipseProblem(80, 60)
    rep = solve(prob, backend="omp", threads=2, return_w=True)
    npy = tmp_path / "w.npy"
    dump.save(npy, rep.w, prob, rep)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "plot_solution.py"), str(npy), "-o",
                          str(tmp_path / "w.ppm")], capture_output=True, text=True, check=True)
    assert (tmp_path / "w.ppm").read_bytes().startswith(b"P6 79 59 255")
    assert "centre line" in out.stdout
    recs = tmp_path / "scale.json"
    recs.write_text("\n".join(json.dumps({"n_gpus": n, "value": v}) for n, v in [(1, 100.0), (2, 190.0), (4, 340.0)]))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "plot_scaling.py"), str(recs), "-o",
                          str(tmp_path / "s.svg")], capture_output=True, text=True, check=True)
    assert "| 4 | 340.0 | 3.40 | 85 % |" in out.stdout
    assert (tmp_path / "s.svg").read_text().startswith("<svg")

"""Reporting: the reference's human-readable lines (parity mode) and JSON.

Reference formats: stage2 ``M=.., N=.. | Iter=.. | Time=%.6f s``
(stage2-mpi/poisson_mpi_decomp.cpp:493-498); stage4 timer block and
``Total Time`` / ``Init`` / ``Solver`` / ``Finalization`` lines
(stage4-mpi+cuda/poisson_mpi_cuda2.cu:968-979, :1026-1034).  The legacy
stage-4 labels are kept verbatim in parity mode ("MPI halo exchange" there
includes the allreduces — here: exchange + allreduce launches + the in-sweep
cross-rank wait, timer ``wait``; the D⁻¹ work is fused into the sweep, so its line
says so instead of printing a zero); the JSON report uses honest category
names.
"""

from __future__ import annotations

import json
import re
from typing import Optional

LEGACY_RESULT_RE = re.compile(r"M=(\d+), N=(\d+) \| Iter=(\d+) \| (?:Total )?Time=([0-9.]+) s")
CONVERGED_RE = re.compile(r"Converged after (\d+) iterations \(\|\|w\(k\+1\)-w\(k\)\|\| < ([0-9.e+-]+)\)\.")


def stage_of(backend: str, ranks: int, threads: int) -> str:
    if backend in ("hip", "hip-group"):
        return "stage4"
    if backend == "serial":
        return "stage0"
    if backend == "omp":
        return "stage1"
    return "stage3" if threads > 1 else "stage2"


def legacy_lines(rep, tol: float = 1e-6) -> str:
    """Reproduce the reference's stdout block for a SolveReport."""
    t = rep.timers
    out = []
    if rep.converged:
        out.append(f"Converged after {rep.iters} iterations (||w(k+1)-w(k)|| < {tol:g}).")
    st = stage_of(rep.backend, rep.ranks, rep.threads)
    if st == "stage4":
        out.append(f"   GPU compute time (Ap + D^{{-1}}r, max over ranks) ~ {t.get('gpu', 0):g} s")
        out.append(f"   Host<->Device copy time (max over ranks)        ~ {t.get('copy', 0):g} s")
        out.append(f"   MPI halo exchange time (max over ranks)         ~ {t.get('halo', 0) + t.get('reduce', 0) + t.get('wait', 0):g} s")
        fused = "n/a (fused into the GPU sweep)"
        out.append(f"   Preconditioner CPU part time (max over ranks)   ~ {fused}")
        dot = fused if t.get("dot_fused", False) else f"{t.get('dot', 0):g} s"
        out.append(f"   Dot products time (max over ranks)              ~ {dot}")
        out.append(f"M={rep.M}, N={rep.N} | Iter={rep.iters} | Total Time={t.get('solver', 0):.6f} s")
        out.append(f"   Init time (program)      ~ {t.get('setup', 0):.6f} s")
        out.append(f"   Solver time (MPI+CUDA)   ~ {t.get('solver', 0):.6f} s")
        out.append(f"   Finalization time        ~ {0.0:.6f} s")
    elif st == "stage0":
        out.append(f"M={rep.M}, N={rep.N} | Iter={rep.iters} | Time={t.get('solver', 0):.4f} s")
    else:
        out.append(f"M={rep.M}, N={rep.N} | Iter={rep.iters} | Time={t.get('solver', 0):.6f} s")
    return "\n".join(out)


def json_report(rep, extra: Optional[dict] = None) -> str:
    d = rep.to_dict()
    if extra:
        d.update(extra)
    return json.dumps(d, sort_keys=True)


def parse_legacy(text: str) -> dict:
    """Parse the reference-format result line(s) back into numbers."""
    m = LEGACY_RESULT_RE.search(text)
    if not m:
        raise ValueError("no result line found")
    out = dict(M=int(m.group(1)), N=int(m.group(2)), iters=int(m.group(3)), time=float(m.group(4)))
    c = CONVERGED_RE.search(text)
    out["converged"] = c is not None
    if c:
        out["tol"] = float(c.group(2))
    return out

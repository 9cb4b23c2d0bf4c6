"""Problem family: -Δu = F on an ellipse embedded in a box, fictitious domain.

Reference (``mxy-kit/poisson-ellipse-openmp-mpi-cuda``, "Variant 9"):
box Π = [-1,1]×[-0.6,0.6] and F = 1 (stage2-mpi/poisson_mpi_decomp.cpp:9-11),
D = {x² + 4y² < 1} (:18-20), ε = max(h1,h2)² (:361), δ = 1e-6 and
max_iter = (M-1)(N-1) (:480-481).  The analytic solution used for accuracy
control is u = (1 - x² - 4y²)/10 (README.md:38-42).

The family generalises the ellipse to cx·x² + cy·y² < 1 with any box / F;
``REFERENCE_PROBLEM`` is the reference's exact configuration and evaluates
bit-identically to it.
"""

from __future__ import annotations

import dataclasses
import math
from typing import Dict

from .._loader import native


@dataclasses.dataclass
class EllipseProblem:
    M: int = 40
    N: int = 40
    A1: float = -1.0
    B1: float = 1.0
    A2: float = -0.6
    B2: float = 0.6
    F: float = 1.0
    # ellipse cx·x² + cy·y² < 1 (semi-axes 1/sqrt(cx), 1/sqrt(cy))
    cx: float = 1.0
    cy: float = 4.0
    tol: float = 1e-6
    max_iter: int = -1
    norm: str = "weighted"  # "weighted" (stage1..4) or "unweighted" (stage0)

    # ---- derived quantities (same formulas as csrc/include/pe/problem.hpp)
    @property
    def h1(self) -> float:
        return (self.B1 - self.A1) / self.M

    @property
    def h2(self) -> float:
        return (self.B2 - self.A2) / self.N

    @property
    def eps(self) -> float:
        h = max(self.h1, self.h2)
        return h * h

    @property
    def iter_cap(self) -> int:
        return self.max_iter if self.max_iter >= 0 else (self.M - 1) * (self.N - 1)

    @property
    def interior_points(self) -> int:
        return (self.M - 1) * (self.N - 1)

    def u_exact(self, x, y):
        """Analytic solution F(1 - cx x² - cy y²)/(2cx + 2cy) inside D (0 outside)."""
        s = self.F / (2.0 * self.cx + 2.0 * self.cy)
        v = s * (1.0 - self.cx * x * x - self.cy * y * y)
        try:
            return v.clamp_min(0.0)  # torch
        except AttributeError:
            import numpy as np

            return np.maximum(v, 0.0)

    def with_grid(self, M: int, N: int) -> "EllipseProblem":
        return dataclasses.replace(self, M=M, N=N)

    def to_native(self):
        nat = native()
        p = nat.Problem()
        p.M, p.N = int(self.M), int(self.N)
        p.A1, p.B1, p.A2, p.B2 = self.A1, self.B1, self.A2, self.B2
        p.F = self.F
        p.cx, p.cy = self.cx, self.cy
        p.sx, p.sy = math.sqrt(self.cx), math.sqrt(self.cy)
        p.tol = self.tol
        p.max_iter = int(self.max_iter)
        p.norm = nat.Norm.Unweighted if self.norm == "unweighted" else nat.Norm.Weighted
        return p


REFERENCE_PROBLEM = EllipseProblem()

# Named configurations: the reference's published grids and the
# BASELINE.json north-star grids.
PRESETS: Dict[str, EllipseProblem] = {
    "ref-40": EllipseProblem(40, 40),
    "ref-400x600": EllipseProblem(400, 600),
    "ref-800x1200": EllipseProblem(800, 1200),
    "ref-1600x2400": EllipseProblem(1600, 2400),
    "ref-2400x3200": EllipseProblem(2400, 3200),
    "stage0-200": EllipseProblem(200, 200, norm="unweighted"),
    "ns-2048": EllipseProblem(2048, 2048),
    "ns-4096": EllipseProblem(4096, 4096),
    "ns-8192": EllipseProblem(8192, 8192),
    "ns-16384": EllipseProblem(16384, 16384),
    # family members beyond the reference
    "circle": EllipseProblem(512, 512, A2=-1.0, B2=1.0, cy=1.0),
    "wide-ellipse": EllipseProblem(1024, 512, A1=-2.0, B1=2.0, A2=-1.0, B2=1.0, cx=0.25, cy=1.0),
}

# Golden iteration counts (δ = 1e-6, w⁰ = 0).  Published: Этап*.pdf; the
# 40×40 / 2048² / 4096² / 8192² values come from the survey's single-rank
# replica of solve_mpi and are reproduced by the CPU oracle.
GOLDEN_ITERS = {
    (40, 40, "weighted"): 50,
    (40, 40, "unweighted"): 61,
    (10, 10, "unweighted"): 17,
    (20, 20, "unweighted"): 31,
    (400, 600, "weighted"): 546,
    (800, 1200, "weighted"): 989,
    (1600, 2400, "weighted"): 1858,
    (2400, 3200, "weighted"): 2449,
    (2048, 2048, "weighted"): 1730,
    (4096, 4096, "weighted"): 3226,
    (8192, 8192, "weighted"): 5889,
    # 16384² (BASELINE.json config 5; no CPU replica run): pinned on 1x MI355X
    # by the classic two-kernel path (reference recurrence, 2 reductions per
    # iteration) and the single sweep, which agree — profiles/r2_pin_16384.txt
    (16384, 16384, "weighted"): 10363,
}

# L2 error in D of the converged solution.
GOLDEN_L2 = {
    (40, 40): 3.68e-3,
    (400, 600): 3.06e-4,
    (800, 1200): 1.92e-4,
    (1600, 2400): 1.78e-4,
    (2400, 3200): 2.10e-4,
    (2048, 2048): 1.67e-4,
    (4096, 4096): 2.71e-4,
    (8192, 8192): 5.88e-4,
    (16384, 16384): 1.4227e-3,  # classic and single sweep: 1.422683e-3 (profiles/r2_pin_16384.txt)
}

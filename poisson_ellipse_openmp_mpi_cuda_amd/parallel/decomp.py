"""2D domain decomposition (Python view of the native implementation).

Reference: choose_process_grid / decompose_2d / neighbour map
(stage2-mpi/poisson_mpi_decomp.cpp:60-111, :246-252).  ``reference`` mode
reproduces the reference's Px = floor(sqrt(P))-then-divisor rule; ``aspect``
mode (default) minimises the per-rank halo cost, preferring contiguous
x-direction rows over strided y-direction columns (e.g. 8 ranks on 8192² →
4×2, 2 ranks on 4096² → 2×1, the BASELINE.json configurations).
"""

from __future__ import annotations

from .._loader import native

MODES = ("aspect", "reference")


def mode_enum(mode: str):
    nat = native()
    if mode not in MODES:
        raise ValueError(f"decomposition mode must be one of {MODES}")
    return nat.DecompMode.Aspect if mode == "aspect" else nat.DecompMode.Reference


def process_grid(P: int, M: int, N: int, mode: str = "aspect"):
    pg = native().choose_process_grid(P, M, N, mode_enum(mode))
    return pg.Px, pg.Py


def block(M: int, N: int, P: int, rank: int, mode: str = "aspect"):
    nat = native()
    pg = nat.choose_process_grid(P, M, N, mode_enum(mode))
    return nat.decompose(M, N, pg, rank)


def blocks(M: int, N: int, P: int, mode: str = "aspect"):
    return [block(M, N, P, r, mode) for r in range(P)]

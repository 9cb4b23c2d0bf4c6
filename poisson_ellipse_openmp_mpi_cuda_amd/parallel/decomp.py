"""2D domain decomposition (Python view of the native implementation).

Reference: choose_process_grid / decompose_2d / neighbour map
(stage2-mpi/poisson_mpi_decomp.cpp:60-111, :246-252).  A decomposition spec
is one of

* ``reference`` — the reference's Px = floor(sqrt(P))-then-divisor rule,
* ``aspect`` (default) — minimum per-rank halo cost, preferring contiguous
  x-direction rows over strided y-direction columns (8 ranks on 8192² →
  4×2, 2 ranks on 4096² → 2×1, the BASELINE.json configurations),
* ``rows`` / ``cols`` — P×1 / 1×P slabs,
* ``device`` — the GPU solver's default: row slabs while every rank keeps
  ≥ 512 rows (one contiguous halo message per side), else ``aspect``,
* ``"<Px>x<Py>"`` — an explicit grid (``"4x2"``).
"""

from __future__ import annotations

from .._loader import native

MODES = ("aspect", "reference", "rows", "cols")
SPECS = MODES + ("device",)


def default_spec(backend: str) -> str:
    """Decomposition used when none is given: "device" for the GPU backends."""
    return "device" if backend in ("hip", "hip-group") else "aspect"


def mode_enum(mode: str):
    nat = native()
    if mode not in MODES:
        raise ValueError(f"decomposition mode must be one of {MODES}")
    return {"aspect": nat.DecompMode.Aspect, "reference": nat.DecompMode.Reference, "rows": nat.DecompMode.Rows,
            "cols": nat.DecompMode.Cols}[mode]


def grid(P: int, M: int, N: int, spec: str = "aspect"):
    """Native ProcessGrid for a decomposition spec (mode name or "PxxPy")."""
    try:
        return native().process_grid_from_spec(spec, P, M, N)
    except Exception as e:  # noqa: BLE001 - surface as ValueError
        raise ValueError(str(e)) from None


def process_grid(P: int, M: int, N: int, mode: str = "aspect"):
    pg = grid(P, M, N, mode)
    return pg.Px, pg.Py


def block(M: int, N: int, P: int, rank: int, mode: str = "aspect"):
    return native().decompose(M, N, grid(P, M, N, mode), rank)


def blocks(M: int, N: int, P: int, mode: str = "aspect"):
    return [block(M, N, P, r, mode) for r in range(P)]

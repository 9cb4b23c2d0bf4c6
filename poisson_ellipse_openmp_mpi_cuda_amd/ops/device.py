"""Single-shot wrappers of the native gfx950 kernels, for numerics tests.

``apply_A_device`` runs the production stencil code path (the same
coefficient classification and arithmetic template the PCG kernels use) on
a caller-supplied field; ``coefficients_device`` returns the a/b/D values the
kernels compute on the fly.  Both use a single-rank block layout
(rows × pitch with a 1-wide halo) and convert to / from the reference's
global (M+1) × (N+1) indexing.
"""

from __future__ import annotations

import numpy as np

from .._loader import native
from ..models.ellipse import EllipseProblem


def _block(prob: EllipseProblem):
    nat = native()
    pg = nat.ProcessGrid()
    pg.Px, pg.Py = 1, 1
    return nat.decompose(prob.M, prob.N, pg, 0)


def to_block(prob: EllipseProblem, g: np.ndarray) -> np.ndarray:
    """Global (M+1, N+1) array → single-rank block field (rows, pitch)."""
    blk = _block(prob)
    f = np.zeros((blk.rows, blk.pitch), dtype=np.float64)
    f[:, : blk.ny + 2] = g[: blk.nx + 2, : blk.ny + 2]
    return f


def from_block(prob: EllipseProblem, f: np.ndarray) -> np.ndarray:
    blk = _block(prob)
    g = np.zeros((prob.M + 1, prob.N + 1), dtype=np.float64)
    g[: blk.nx + 2, : blk.ny + 2] = f[:, : blk.ny + 2]
    return g


def apply_A_device(prob: EllipseProblem, p_global: np.ndarray) -> np.ndarray:
    nat = native()
    blk = _block(prob)
    out = nat.device_apply_A(prob.to_native(), blk, np.ascontiguousarray(to_block(prob, p_global)))
    g = from_block(prob, np.asarray(out))
    g[0, :] = g[-1, :] = 0
    g[:, 0] = g[:, -1] = 0
    return g


def coefficients_device(prob: EllipseProblem):
    """(a, b, D) as the kernels see them, in global (M+1, N+1) indexing
    (valid for i ∈ [0, M], j ∈ [0, N]; D is meaningful on interior nodes)."""
    nat = native()
    blk = _block(prob)
    a, b, D = nat.device_coefficients(prob.to_native(), blk)
    return from_block(prob, np.asarray(a)), from_block(prob, np.asarray(b)), from_block(prob, np.asarray(D))

"""Solution dumps (the reference plots w at 800×1200 with an external script
that is not in the repository: Этап3.pdf p.9).  ``save`` writes the interior
of w as ``.npy`` plus a JSON sidecar (grid, box, iteration count, errors);
``write_pgm`` renders a grey-scale heat map without any plotting library.
"""

from __future__ import annotations

import json
from pathlib import Path

import numpy as np


def save(path, w: np.ndarray, prob, rep=None) -> None:
    path = Path(path)
    np.save(path, np.ascontiguousarray(w))
    meta = dict(M=prob.M, N=prob.N, box=[prob.A1, prob.B1, prob.A2, prob.B2], cx=prob.cx, cy=prob.cy, F=prob.F,
                layout="w[i-1, j-1] for interior node (x_i, y_j), i=1..M-1, j=1..N-1")
    if rep is not None:
        meta.update(iters=rep.iters, l2_err=rep.l2_err, max_err=rep.max_err, backend=rep.backend)
    path.with_suffix(".json").write_text(json.dumps(meta, indent=1))


def load(path):
    path = Path(path)
    w = np.load(path, allow_pickle=False)
    meta = json.loads(path.with_suffix(".json").read_text()) if path.with_suffix(".json").exists() else {}
    return w, meta


def write_pgm(path, w: np.ndarray, max_side: int = 1024) -> None:
    """Grey-scale image of w (x → columns, y up), downsampled to ≤ max_side."""
    a = np.asarray(w, dtype=np.float64).T[::-1]  # rows = y (top = +y), cols = x
    sy = max(1, int(np.ceil(a.shape[0] / max_side)))
    sx = max(1, int(np.ceil(a.shape[1] / max_side)))
    a = a[::sy, ::sx]
    lo, hi = float(a.min()), float(a.max())
    img = np.zeros_like(a) if hi <= lo else (a - lo) / (hi - lo)
    data = (img * 255.0 + 0.5).astype(np.uint8)
    with open(path, "wb") as f:
        f.write(f"P5\n{data.shape[1]} {data.shape[0]}\n255\n".encode())
        f.write(data.tobytes())

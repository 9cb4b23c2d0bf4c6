#!/usr/bin/env python3
"""Colour heat map of a solution dump (``--dump w.npy``) as a binary PPM, plus
a centre-line profile against the analytic solution — the reference's
800×1200 heat map (Этап3.pdf p.9) without a plotting library.

    python -m poisson_ellipse_openmp_mpi_cuda_amd --backend hip --dump w.npy 800 1200
    python tools/plot_solution.py w.npy -o w.ppm
"""

import argparse
import json
import sys
from pathlib import Path

import numpy as np


def colormap(t):
    # blue → cyan → yellow → red
    stops = np.array([[0.0, 0.0, 0.5], [0.0, 0.8, 1.0], [1.0, 1.0, 0.0], [0.8, 0.0, 0.0]])
    x = np.clip(t, 0, 1) * (len(stops) - 1)
    i = np.minimum(x.astype(int), len(stops) - 2)
    f = (x - i)[..., None]
    return stops[i] * (1 - f) + stops[i + 1] * f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npy")
    ap.add_argument("-o", "--out", default="w.ppm")
    ap.add_argument("--max-side", type=int, default=1200)
    a = ap.parse_args()
    w = np.load(a.npy, allow_pickle=False)
    meta_p = Path(a.npy).with_suffix(".json")
    meta = json.loads(meta_p.read_text()) if meta_p.exists() else {}
    img = w.T[::-1]  # rows = y (top = +y), columns = x
    s = max(1, int(np.ceil(max(img.shape) / a.max_side)))
    img = img[::s, ::s]
    lo, hi = float(img.min()), float(img.max())
    rgb = (colormap((img - lo) / (hi - lo if hi > lo else 1.0)) * 255 + 0.5).astype(np.uint8)
    with open(a.out, "wb") as f:
        f.write(f"P6 {rgb.shape[1]} {rgb.shape[0]} 255\n".encode())
        f.write(rgb.tobytes())
    print(f"wrote {a.out}: {rgb.shape[1]}x{rgb.shape[0]}, w in [{lo:.4g}, {hi:.4g}]")
    if meta:
        M, N = meta["M"], meta["N"]
        A1, B1, A2, B2 = meta["box"]
        cx, cy, F = meta.get("cx", 1.0), meta.get("cy", 4.0), meta.get("F", 1.0)
        i = M // 2
        x = A1 + i * (B1 - A1) / M
        y = A2 + np.arange(1, N) * (B2 - A2) / N
        u = np.where(cx * x * x + cy * y * y < 1, F * (1 - cx * x * x - cy * y * y) / (2 * cx + 2 * cy), 0.0)
        err = np.abs(w[i - 1] - u).max()
        print(f"centre line x = {x:.4f}: max |w - u| = {err:.3e} (peak w = {w[i - 1].max():.5f}, u = {u.max():.5f})")
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""Independent PyTorch fp64 oracle of the fictitious-domain operator and PCG.

A vectorised re-statement of the reference numerics (fic_reg_local,
mat_A_local, mat_D, dot_local, solve_mpi in
stage2-mpi/poisson_mpi_decomp.cpp:124-460) on whole-grid tensors, used by the
tests as an oracle for the native CPU backends and the gfx950 kernels.  It
runs on any torch device ("cpu" here, "cuda" = HIP on the GPU box).

Arrays use the reference's global indexing: shape (M+1, N+1), index [i, j]
for node (x_i, y_j); interior unknowns are [1:M, 1:N]; the box boundary is
held at 0 (Dirichlet).
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch

from ..models.ellipse import EllipseProblem


def _div(a: torch.Tensor, s: float) -> torch.Tensor:
    """a / s, correctly rounded.  (PyTorch's CPU `tensor / python_scalar`
    multiplies by the reciprocal, which differs from IEEE division in the last
    bit — enough to break bitwise parity with the reference formulas.)"""
    return a / torch.full_like(a, s)


def _grid(prob: EllipseProblem, device, dtype=torch.float64):
    h1, h2 = prob.h1, prob.h2
    i = torch.arange(0, prob.M + 1, device=device, dtype=dtype)
    j = torch.arange(0, prob.N + 1, device=device, dtype=dtype)
    x = prob.A1 + i * h1
    y = prob.A2 + j * h2
    return x, y


def _face_coef_np(l, h, eps):
    import numpy as np

    blend = (l / h) + (1.0 - l / h) / eps
    out = np.where(l < 1e-9, 1.0 / eps, blend)
    return np.where(np.abs(l - h) < 1e-9, 1.0, out)


def assemble(prob: EllipseProblem, device="cpu"):
    """Coefficients a, b (shape (M+1, N+1); row/col 0 unused) and RHS B.

    Built with numpy (hardware IEEE sqrt / division: bit-identical to the
    reference's C++ fic_reg) and moved to `device`; PyTorch's CPU sqrt and
    scalar division are not always correctly rounded.
    """
    import numpy as np

    h1, h2, eps = prob.h1, prob.h2, prob.eps
    sx, sy = math.sqrt(prob.cx), math.sqrt(prob.cy)
    x = prob.A1 + np.arange(0, prob.M + 1, dtype=np.float64) * h1
    y = prob.A2 + np.arange(0, prob.N + 1, dtype=np.float64) * h2
    X = x[:, None] + np.zeros((1, y.size))
    Y = y[None, :] + np.zeros((x.size, 1))
    with np.errstate(invalid="ignore"):
        # vertical face at x_i - h1/2 over [y_j - h2/2, y_j + h2/2]
        c = X - 0.5 * h1
        half = np.sqrt(np.maximum(0.0, (1.0 - prob.cx * c * c) / prob.cy))
        la = np.maximum(0.0, np.minimum(Y + 0.5 * h2, half) - np.maximum(Y - 0.5 * h2, -half))
        la = np.where(np.abs(sx * c) >= 1.0, 0.0, la)
        # horizontal face at y_j - h2/2 over [x_i - h1/2, x_i + h1/2]
        c2 = Y - 0.5 * h2
        half2 = np.sqrt(np.maximum(0.0, (1.0 - prob.cy * c2 * c2) / prob.cx))
        lb = np.maximum(0.0, np.minimum(X + 0.5 * h1, half2) - np.maximum(X - 0.5 * h1, -half2))
        lb = np.where(np.abs(sy * c2) >= 1.0, 0.0, lb)
    a = _face_coef_np(la, h2, eps)
    b = _face_coef_np(lb, h1, eps)
    inside = (prob.cx * X * X + prob.cy * Y * Y) < 1.0
    B = np.where(inside, prob.F, 0.0)
    B[0, :] = B[-1, :] = 0.0
    B[:, 0] = B[:, -1] = 0.0
    t = lambda v: torch.from_numpy(np.ascontiguousarray(v)).to(device)  # noqa: E731
    return t(a), t(b), t(B)


def apply_A(p, a, b, h1, h2):
    """(A p) on interior nodes; boundary rows/cols of the result are 0."""
    out = torch.zeros_like(p)
    pc = p[1:-1, 1:-1]
    Ax = (-1.0 / h1) * (_div(a[2:, 1:-1] * (p[2:, 1:-1] - pc), h1) - _div(a[1:-1, 1:-1] * (pc - p[:-2, 1:-1]), h1))
    Ay = (-1.0 / h2) * (_div(b[1:-1, 2:] * (p[1:-1, 2:] - pc), h2) - _div(b[1:-1, 1:-1] * (pc - p[1:-1, :-2]), h2))
    out[1:-1, 1:-1] = Ax + Ay
    return out


def diag(a, b, h1, h2):
    """Jacobi diagonal D on interior nodes (0 elsewhere)."""
    D = torch.zeros_like(a)
    D[1:-1, 1:-1] = _div(a[2:, 1:-1] + a[1:-1, 1:-1], h1 * h1) + _div(b[1:-1, 2:] + b[1:-1, 1:-1], h2 * h2)
    return D


def apply_Dinv(r, D):
    z = torch.zeros_like(r)
    m = D != 0
    z[m] = r[m] / D[m]
    return z


def dot(u, v, h1, h2):
    return float((u[1:-1, 1:-1] * v[1:-1, 1:-1]).sum()) * h1 * h2


@dataclass
class TorchPCGResult:
    iters: int
    converged: bool
    w: torch.Tensor
    l2_err: float
    max_err: float
    history: list


def pcg(prob: EllipseProblem, device="cpu", w0: Optional[torch.Tensor] = None, max_iter: Optional[int] = None,
        keep_history: bool = False) -> TorchPCGResult:
    """Reference-algorithm Jacobi PCG (stage2 solve_mpi order of operations)."""
    a, b, B = assemble(prob, device)
    h1, h2 = prob.h1, prob.h2
    D = diag(a, b, h1, h2)
    w = torch.zeros_like(B) if w0 is None else w0.clone()
    r = B - apply_A(w, a, b, h1, h2)
    r[0, :] = r[-1, :] = 0
    r[:, 0] = r[:, -1] = 0
    z = apply_Dinv(r, D)
    p = z.clone()
    zr_old = dot(z, r, h1, h2)
    cap = prob.iter_cap if max_iter is None else max_iter
    hist = []
    converged = False
    k = 0
    for k in range(1, cap + 1):
        Ap = apply_A(p, a, b, h1, h2)
        den = dot(Ap, p, h1, h2)
        if abs(den) < 1e-15:
            break
        alpha = zr_old / den
        dw = alpha * p
        w = w + dw
        r = r - alpha * Ap
        z = apply_Dinv(r, D)
        zr_new = dot(z, r, h1, h2)
        d2 = float((dw[1:-1, 1:-1] ** 2).sum())
        diff = math.sqrt(d2 * h1 * h2) if prob.norm == "weighted" else math.sqrt(d2)
        if keep_history:
            hist.append(diff)
        if diff < prob.tol:
            converged = True
            break
        beta = zr_new / zr_old
        zr_old = zr_new
        p = z + beta * p
    l2, mx = error_vs_analytic(prob, w)
    return TorchPCGResult(k, converged, w, l2, mx, hist)


@dataclass
class SingleSweepState:
    iters: int
    sums: list    # per iteration k = 0 (S_0) .. K: the 7 unweighted sums of sweep k
    alpha: list   # α_k, β_k for k = 1 .. K
    beta: list
    r: torch.Tensor
    p: torch.Tensor
    w: torch.Tensor


def single_sweep(prob: EllipseProblem, iters: int, device="cpu") -> SingleSweepState:
    """The single-reduction recurrence of the device sweep kernels
    (csrc/hip/fused.hip header, sweep_scalars), on the reference operator.

    Sweep 0 (S_0): z₀ = D⁻¹r₀, q₀ = A z₀ and their sums.  Sweep k ≥ 1, from
    sweep k-1's sums R = {(r,z) (z,q) (z,s) (p,s) (z,z) (z,p) (p,p)}:
        g = R₀h², β = g/g_prev (0 at k = 1), den = (R₁ + 2βR₂ + β²R₃)h², α = g/den
        p = z + βp, s = Ap, w += αp, r -= αs, z = D⁻¹r, q = Az → sums of sweep k.
    Algebraically the reference PCG (stage2-mpi/poisson_mpi_decomp.cpp:400-457)."""
    a, b, B = assemble(prob, device)
    h1, h2 = prob.h1, prob.h2
    hh = h1 * h2
    D = diag(a, b, h1, h2)
    inner = lambda u, v: float((u[1:-1, 1:-1] * v[1:-1, 1:-1]).sum())  # noqa: E731  (unweighted)
    r = B.clone()
    p = torch.zeros_like(B)
    w = torch.zeros_like(B)
    s = torch.zeros_like(B)
    z = apply_Dinv(r, D)
    q = apply_A(z, a, b, h1, h2)
    sums = [[inner(r, z), inner(z, q), inner(z, s), inner(p, s), inner(z, z), inner(z, p), inner(p, p)]]
    alphas, betas = [], []
    gprev = 0.0
    for k in range(1, iters + 1):
        R = sums[-1]
        g = R[0] * hh
        beta = 0.0 if k == 1 else g / gprev
        den = R[1] * hh + 2.0 * beta * (R[2] * hh) + beta * beta * (R[3] * hh)
        alpha = g / den
        p = z + beta * p
        s = apply_A(p, a, b, h1, h2)
        w = w + alpha * p
        r = r - alpha * s
        z = apply_Dinv(r, D)
        q = apply_A(z, a, b, h1, h2)
        sums.append([inner(r, z), inner(z, q), inner(z, s), inner(p, s), inner(z, z), inner(z, p), inner(p, p)])
        alphas.append(alpha)
        betas.append(beta)
        gprev = g
    return SingleSweepState(iters, sums, alphas, betas, r, p, w)


@dataclass
class TwoStepState:
    sweeps: int
    sums: list    # per sweep j = 0 (S_0) .. J: the 20 unweighted sums (csrc/hip/fused2.hip layout)
    alpha: list   # (α₁, α₂) per sweep j ≥ 1
    beta: list    # (β₁, β₂)
    diff: list    # (‖Δw‖ of iteration 2j-1, of 2j)
    r: torch.Tensor
    p: torch.Tensor
    w: torch.Tensor


def two_step_sums(r, p, a, b, h1, h2, Dinv):
    """The 20 sums of the basis around (r, p) (fused2.hip, sweep2_scalars)."""
    inner = lambda u, v: float((u[1:-1, 1:-1] * v[1:-1, 1:-1]).sum())  # noqa: E731  (unweighted)
    A = lambda u: apply_A(u, a, b, h1, h2)  # noqa: E731
    z = Dinv * r
    s = A(p)
    q = A(z)
    u = Dinv * q
    v = Dinv * s
    Au, Av = A(u), A(v)
    return [inner(r, z), inner(z, q), inner(z, s), inner(p, s), inner(q, u), inner(u, s), inner(s, v),
            inner(u, Au), inner(u, Av), inner(v, Av), inner(z, z), inner(z, p), inner(z, u), inner(z, v),
            inner(p, p), inner(p, u), inner(p, v), inner(u, u), inner(u, v), inner(v, v)]


def two_step_scalars(R, gprev: float, K: int, hh: float, weighted: bool = True):
    """(g1, β1, α1, ‖Δw‖1, g2, β2, α2, ‖Δw‖2) of the sweep covering iterations
    K+1, K+2 from the previous sweep's sums R — the device's sweep2_scalars."""
    g1 = R[0] * hh
    b1 = 0.0 if K == 0 else g1 / gprev
    den1 = (R[1] + 2.0 * b1 * R[2] + b1 * b1 * R[3]) * hh
    a1 = g1 / den1
    pn1 = max(R[10] + 2.0 * b1 * R[11] + b1 * b1 * R[14], 0.0)
    d1 = abs(a1) * math.sqrt(pn1 * hh if weighted else pn1)
    g2 = (R[0] - 2.0 * a1 * (R[1] + b1 * R[2]) + a1 * a1 * (R[4] + 2.0 * b1 * R[5] + b1 * b1 * R[6])) * hh
    b2 = g2 / g1
    c = [1.0 + b2, b1 * b2, -a1, -a1 * b1]
    G = [[R[1], R[2], R[4], R[5]], [R[2], R[3], R[5], R[6]], [R[4], R[5], R[7], R[8]], [R[5], R[6], R[8], R[9]]]
    P = [[R[10], R[11], R[12], R[13]], [R[11], R[14], R[15], R[16]], [R[12], R[15], R[17], R[18]],
         [R[13], R[16], R[18], R[19]]]
    qf = lambda m: sum(c[i] * c[j] * m[i][j] for i in range(4) for j in range(4))  # noqa: E731
    den2 = qf(G) * hh
    a2 = g2 / den2
    pn2 = max(qf(P), 0.0)
    d2 = abs(a2) * math.sqrt(pn2 * hh if weighted else pn2)
    return g1, b1, a1, d1, g2, b2, a2, d2, den1, den2


def two_step(prob: EllipseProblem, sweeps: int, device="cpu") -> TwoStepState:
    """The two-iterations-per-sweep recurrence of csrc/hip/fused2.hip on the
    reference operator (divisions): S_0 (the sums around r₀ = B, p₀ = 0),
    then `sweeps` sweeps, each advancing iterations K+1 and K+2 with scalars
    from the previous sweep's 20 sums.  Algebraically the reference PCG
    (stage2-mpi/poisson_mpi_decomp.cpp:400-457), two iterations at a time."""
    a, b, B = assemble(prob, device)
    h1, h2 = prob.h1, prob.h2
    hh = h1 * h2
    D = diag(a, b, h1, h2)
    Dinv = torch.zeros_like(D)
    m = D != 0
    Dinv[m] = 1.0 / D[m]
    A = lambda u: apply_A(u, a, b, h1, h2)  # noqa: E731
    r = B.clone()
    p = torch.zeros_like(B)
    w = torch.zeros_like(B)
    sums = [two_step_sums(r, p, a, b, h1, h2, Dinv)]
    alphas, betas, diffs = [], [], []
    gprev = 0.0
    for j in range(1, sweeps + 1):
        K = 2 * (j - 1)
        g1, b1, a1, d1, g2, b2, a2, d2, _, _ = two_step_scalars(sums[-1], gprev, K, hh, prob.norm == "weighted")
        z = Dinv * r
        p1 = z + b1 * p
        r1 = r - a1 * A(p1)
        z1 = Dinv * r1
        p2 = z1 + b2 * p1
        r = r1 - a2 * A(p2)
        w = w + a1 * p1 + a2 * p2
        p = p2
        gprev = g2
        sums.append(two_step_sums(r, p, a, b, h1, h2, Dinv))
        alphas.append((a1, a2))
        betas.append((b1, b2))
        diffs.append((d1, d2))
    return TwoStepState(sweeps, sums, alphas, betas, diffs, r, p, w)


@dataclass
class ThreeStepState:
    sweeps: int
    sums: list    # per sweep j = 0 (S_0) .. J: the 19 unweighted sums (csrc/hip/fused3.hip layout)
    alpha: list   # (α₁, α₂, α₃) per sweep j ≥ 1
    beta: list    # (β₁, β₂, β₃)
    diff: list    # ‖Δw‖ of its three iterations (late: from the sweep's own ‖p_i‖² sums)
    r: torch.Tensor
    p: torch.Tensor
    w: torch.Tensor


def three_step_moments(r, p, a, b, h1, h2, Dinv):
    """The 16 D-moments of the basis around (r, p) (fused3.hip sums 0..15)."""
    inner = lambda u, v: float((u[1:-1, 1:-1] * v[1:-1, 1:-1]).sum())  # noqa: E731  (unweighted)
    A = lambda u: apply_A(u, a, b, h1, h2)  # noqa: E731
    z = Dinv * r
    s = A(p)
    q = A(z)
    u, v = Dinv * q, Dinv * s
    Au, Av = A(u), A(v)
    uu, vv = Dinv * Au, Dinv * Av
    Auu, Avv = A(uu), A(vv)
    return [inner(r, z), inner(z, q), inner(q, u), inner(u, Au), inner(Au, uu), inner(uu, Auu),
            inner(z, s), inner(q, v), inner(u, Av), inner(Au, vv), inner(uu, Avv),
            inner(p, s), inner(s, v), inner(v, Av), inner(Av, vv), inner(vv, Avv)]


def _mform(xz, xp, mzz, mzp, mpp, sh):
    s = 0.0
    for i in range(3):
        for j in range(3):
            n = i + j + sh
            s += xz[i] * (xz[j] * mzz[n] + 2.0 * xp[j] * mzp[n]) + xp[i] * xp[j] * mpp[n]
    return s


def three_step_scalars(R, gprev: float, K: int, hh: float, lim: int = 3):
    """[(g, β, α)] of the (up to lim) iterations of the sweep after K from the
    previous sweep's sums R — fused3.hip's sweep3_scalars (None past a breakdown)."""
    mzz = R[0:6]
    mzp = [0.0] + list(R[6:11])
    mpp = [0.0] + list(R[11:16])
    zz, zp = [1.0, 0.0, 0.0], [0.0, 0.0, 0.0]
    pz, pp = [0.0, 0.0, 0.0], [1.0, 0.0, 0.0]
    g = _mform(zz, zp, mzz, mzp, mpp, 0) * hh
    out = []
    for i in range(lim):
        beta = 0.0 if K + i == 0 else g / gprev
        pz = [zz[q] + beta * pz[q] for q in range(3)]
        pp = [zp[q] + beta * pp[q] for q in range(3)]
        den = _mform(pz, pp, mzz, mzp, mpp, 1) * hh
        if not math.isfinite(den) or abs(den) < 1e-15:
            break
        alpha = g / den
        out.append((g, beta, alpha))
        gprev = g
        if i + 1 < lim:
            zz[2] -= alpha * pz[1]
            zz[1] -= alpha * pz[0]
            zp[2] -= alpha * pp[1]
            zp[1] -= alpha * pp[0]
            g = _mform(zz, zp, mzz, mzp, mpp, 0) * hh
    return out


def three_step(prob: EllipseProblem, sweeps: int, device="cpu") -> ThreeStepState:
    """The three-iterations-per-sweep recurrence of csrc/hip/fused3.hip on the
    reference operator (divisions): S_0, then `sweeps` full sweeps, each
    advancing iterations K+1..K+3 with scalars from the previous sweep's 16
    moments; the sweep's own ‖p_i‖² give the (late) ‖Δw‖.  Algebraically the
    reference PCG (stage2-mpi/poisson_mpi_decomp.cpp:400-457)."""
    a, b, B = assemble(prob, device)
    h1, h2 = prob.h1, prob.h2
    hh = h1 * h2
    D = diag(a, b, h1, h2)
    Dinv = torch.zeros_like(D)
    m = D != 0
    Dinv[m] = 1.0 / D[m]
    A = lambda u: apply_A(u, a, b, h1, h2)  # noqa: E731
    inner = lambda u, v: float((u[1:-1, 1:-1] * v[1:-1, 1:-1]).sum())  # noqa: E731
    weighted = prob.norm == "weighted"
    r = B.clone()
    p = torch.zeros_like(B)
    w = torch.zeros_like(B)
    sums = [three_step_moments(r, p, a, b, h1, h2, Dinv) + [0.0, 0.0, 0.0]]
    alphas, betas, diffs = [], [], []
    gprev = 0.0
    for j in range(1, sweeps + 1):
        K = 3 * (j - 1)
        sc = three_step_scalars(sums[-1], gprev, K, hh)
        assert len(sc) == 3, "breakdown inside the reference sweeps"
        norms = []
        for (g, beta, alpha) in sc:
            p = Dinv * r + beta * p
            norms.append(inner(p, p))
            r = r - alpha * A(p)
            w = w + alpha * p
            gprev = g
        alphas.append(tuple(x[2] for x in sc))
        betas.append(tuple(x[1] for x in sc))
        diffs.append(tuple(abs(x[2]) * math.sqrt(n * hh if weighted else n) for x, n in zip(sc, norms)))
        sums.append(three_step_moments(r, p, a, b, h1, h2, Dinv) + norms)
    return ThreeStepState(sweeps, sums, alphas, betas, diffs, r, p, w)


def error_vs_analytic(prob: EllipseProblem, w: torch.Tensor):
    """(L2 error in D, h-weighted; max error in D) against u = F(1-cx x²-cy y²)/(2cx+2cy)."""
    x, y = _grid(prob, w.device)
    X = x[:, None]
    Y = y[None, :]
    inside = (prob.cx * X * X + prob.cy * Y * Y) < 1.0
    u = prob.F / (2.0 * prob.cx + 2.0 * prob.cy) * (1.0 - prob.cx * X * X - prob.cy * Y * Y)
    e = torch.where(inside, w - u, torch.zeros_like(w))[1:-1, 1:-1]
    return math.sqrt(float((e * e).sum()) * prob.h1 * prob.h2), float(e.abs().max())

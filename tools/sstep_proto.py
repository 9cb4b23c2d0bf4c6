"""s-step (s = 2, 3) Jacobi-PCG in the moment form a device sweep would use:
iteration count check against the golden values before committing a kernel
to it.

Each sweep advances iterations K+1..K+s from scalars that are quadratic forms
in D-moments  mu_k(x, y) = (x, D M^k y), M = D^-1 A, of z = D^-1 r_K and p_K
(k = 0..2s-1), computed by the PREVIOUS sweep as single dot products of
vectors it forms anyway:
    zz: (r,z) (z,q) (q,u) (u,Au) (Au,uu) (uu,A uu)       q = Az, u = D^-1 q, uu = D^-1 Au
    zp:       (z,s) (q,v) (u,Av) (Av... )                 s = Ap, v = D^-1 s, vv = D^-1 Av
    pp:       (p,s) (s,v) (v,Av) (Av,vv) (vv,A vv)
The stop test of iteration K+i (|alpha| ||p_i||) uses ||p_i||^2 summed in the
sweep that forms p_i ("late" norms): a stop before the sweep's last
iteration is resolved after it (the device subtracts the extra updates).

    python tools/sstep_proto.py 3 [cpu|cuda] [grids...]    e.g. 400x600 800x1200
"""
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from poisson_ellipse_openmp_mpi_cuda_amd import EllipseProblem  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.models.ellipse import GOLDEN_ITERS  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.ops.torch_ref import apply_A, assemble, diag  # noqa: E402


def moments(r, p, A, Dinv, inner, s):
    """mu[x][k] for x in (zz, zp, pp), k = 0 .. 2s-1 (NaN where not formed).
    s <= 3: the pairs fused3.hip forms; larger s: (M^a x, D M^b y), a = k // 2."""
    z = Dinv * r
    sv = A(p)
    nan = float("nan")
    if s > 3:
        D = torch.zeros_like(Dinv)
        m = Dinv != 0
        D[m] = 1.0 / Dinv[m]
        Mz, Mp = [z], [p]
        for _ in range(s):
            Mz.append(Dinv * A(Mz[-1]))
            Mp.append(Dinv * A(Mp[-1]))
        mu = {"zz": [], "zp": [nan], "pp": [nan]}
        for k in range(2 * s):
            a, b = k // 2, k - k // 2
            mu["zz"].append(inner(Mz[a], D * Mz[b]) if k else inner(r, z))
            if k:
                mu["zp"].append(inner(Mz[a], D * Mp[b]))
                mu["pp"].append(inner(Mp[a], D * Mp[b]))
        return mu
    q = A(z)
    u = Dinv * q
    v = Dinv * sv
    zz = [inner(r, z), inner(z, q), inner(q, u)]
    zp = [nan, inner(z, sv), inner(q, v)]
    pp = [nan, inner(p, sv), inner(sv, v)]
    Au, Av = A(u), A(v)
    zz.append(inner(u, Au))
    zp.append(inner(u, Av))
    pp.append(inner(v, Av))
    if s >= 3:
        uu, vv = Dinv * Au, Dinv * Av
        Auu, Avv = A(uu), A(vv)
        zz += [inner(Au, uu), inner(uu, Auu)]
        zp += [inner(Au, vv), inner(uu, Avv)]
        pp += [inner(Av, vv), inner(vv, Avv)]
    return {"zz": zz, "zp": zp, "pp": pp}


def dform(cx, cy, mu, shift):
    """(x, D M^shift y) for x, y given as coefficients over (M^a z, M^a p)."""
    s = len(cx[0])
    acc = 0.0
    for a in range(s):
        for b in range(s):
            k = a + b + shift
            t = cx[0][a] * cy[0][b]
            if t != 0.0:
                acc += t * mu["zz"][k]
            t = cx[0][a] * cy[1][b] + cx[1][a] * cy[0][b]
            if t != 0.0:
                acc += t * mu["zp"][k]
            t = cx[1][a] * cy[1][b]
            if t != 0.0:
                acc += t * mu["pp"][k]
    return acc


def shiftM(c):
    return [[0.0] + c[0][:-1], [0.0] + c[1][:-1]]


def sstep_solve(prob, s, device="cpu"):
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
    cap = prob.iter_cap
    r = B.clone()
    p = torch.zeros_like(B)
    mu = moments(r, p, A, Dinv, inner, s)
    gprev, K = 0.0, 0
    while True:
        zc = [[1.0] + [0.0] * (s - 1), [0.0] * s]
        pc = [[0.0] * s, [1.0] + [0.0] * (s - 1)]
        g = dform(zc, zc, mu, 0) * hh
        al, be, nb = [], [], s
        for i in range(s):
            beta = 0.0 if K + i == 0 else g / gprev
            pc = [[zc[t][j] + beta * pc[t][j] for j in range(s)] for t in range(2)]
            den = dform(pc, pc, mu, 1) * hh
            if not math.isfinite(den) or abs(den) < 1e-15:
                nb = i
                break
            alpha = g / den
            al.append(alpha)
            be.append(beta)
            gprev = g
            if i + 1 < s:
                Mp = shiftM(pc)
                zc = [[zc[t][j] - alpha * Mp[t][j] for j in range(s)] for t in range(2)]
                g = dform(zc, zc, mu, 0) * hh
        # the sweep: nb iterations, late norms
        zz = Dinv * r
        stop = None
        for j in range(nb):
            p = zz + be[j] * p
            n2 = inner(p, p)
            r = r - al[j] * A(p)
            zz = Dinv * r
            diff = abs(al[j]) * math.sqrt(n2 * hh if weighted else n2)
            k = K + j + 1
            if stop is None and (diff < prob.tol or k >= cap):
                stop = (k, "conv" if diff < prob.tol else "cap")
        if stop is not None:
            return stop
        if nb < s:
            return (K + nb + 1, "breakdown")
        K += s
        mu = moments(r, p, A, Dinv, inner, s)


if __name__ == "__main__":
    s = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = sys.argv[2] if len(sys.argv) > 2 else "cpu"
    grids = sys.argv[3:] or ["40x40", "400x600", "800x1200"]
    bad = 0
    for gspec in grids:
        norm = "weighted"
        if gspec.endswith("u"):
            norm, gspec = "unweighted", gspec[:-1]
        M, N = (int(v) for v in gspec.split("x"))
        t = time.time()
        it, why = sstep_solve(EllipseProblem(M, N, norm=norm), s, dev)
        want = GOLDEN_ITERS.get((M, N, norm))
        ok = want is None or it == want
        bad += not ok
        print(f"s={s} {M}x{N} {norm}: {it} ({why}) golden {want} {'OK' if ok else 'MISMATCH'} {time.time() - t:.1f}s",
              flush=True)
    sys.exit(1 if bad else 0)

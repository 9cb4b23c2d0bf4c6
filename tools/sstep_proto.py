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


def sstep_solve(prob, s, device="cpu", init="zero", seed=1234, stats=None):
    """Iteration count and stop reason.  stats (a dict) receives the largest
    relative deviation of the moment-form alpha / beta from the same scalars
    computed directly on the sweep's vectors, and the final recurrence gap
    ||B - A w - r|| / ||r|| (what the device's end-of-solve check measures)."""
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
    w = torch.zeros_like(B)
    if init == "random":  # w0 = amp * uniform(-1, 1) on the interior (parity unpinned: the reference has w0 = 0)
        g = torch.Generator(device="cpu").manual_seed(seed)
        w[1:-1, 1:-1] = (0.05 * (2 * torch.rand(w[1:-1, 1:-1].shape, generator=g, dtype=torch.float64) - 1)).to(device)
    r = B - A(w)
    r[0, :] = 0
    r[-1, :] = 0
    r[:, 0] = 0
    r[:, -1] = 0
    p = torch.zeros_like(B)
    mu = moments(r, p, A, Dinv, inner, s)
    gprev, K = 0.0, 0
    dev_a = dev_b = 0.0
    gdir_prev = None
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
            if stats is not None:  # the same scalars from the vectors themselves
                gdir = inner(r, zz) * hh
                if gdir_prev is not None and K + j > 0:
                    bd = gdir / gdir_prev
                    dev_b = max(dev_b, abs(be[j] - bd) / max(abs(bd), 1e-300))
                gdir_prev = gdir
            p = zz + be[j] * p
            n2 = inner(p, p)
            Ap = A(p)
            if stats is not None:
                ad = gdir / (inner(Ap, p) * hh)
                dev_a = max(dev_a, abs(al[j] - ad) / max(abs(ad), 1e-300))
            r = r - al[j] * Ap
            w = w + al[j] * p
            zz = Dinv * r
            diff = abs(al[j]) * math.sqrt(n2 * hh if weighted else n2)
            k = K + j + 1
            if stop is None and (diff < prob.tol or k >= cap):
                stop = (k, "conv" if diff < prob.tol else "cap")
        if stop is not None or nb < s:
            if stats is not None:
                rho = B - A(w)
                dr = rho - r
                stats.update(alpha_dev=dev_a, beta_dev=dev_b,
                             gap=math.sqrt(inner(dr, dr) / max(inner(r, r), 1e-300)))
            # (the device stops w at the stop iteration; here w ran to the end of the sweep: the gap is
            # measured on the pair (w, r) of the same iterate either way)
            return stop if stop is not None else (K + nb + 1, "breakdown")
        K += s
        if K % 1500 < s:  # (progress: a long GPU run must not look hung)
            print(f"  ... iteration {K}", file=sys.stderr, flush=True)
        mu = moments(r, p, A, Dinv, inner, s)


if __name__ == "__main__":
    s = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = sys.argv[2] if len(sys.argv) > 2 else "cpu"
    grids = sys.argv[3:] or ["40x40", "400x600", "800x1200"]
    bad = 0
    for gspec in grids:
        # suffixes: u = unweighted norm, r = random init w0 (no golden: reported only)
        norm, init = "weighted", "zero"
        while gspec[-1] in "ur":
            if gspec.endswith("u"):
                norm = "unweighted"
            else:
                init = "random"
            gspec = gspec[:-1]
        M, N = (int(v) for v in gspec.split("x"))
        t = time.time()
        st = {}
        it, why = sstep_solve(EllipseProblem(M, N, norm=norm), s, dev, init=init, stats=st)
        want = GOLDEN_ITERS.get((M, N, norm)) if init == "zero" else None
        ok = want is None or it == want
        bad += not ok
        print(f"s={s} {M}x{N} {norm} w0={init}: {it} ({why}) golden {want} {'OK' if ok else 'MISMATCH'}  "
              f"max rel dev alpha {st.get('alpha_dev', float('nan')):.2e} beta {st.get('beta_dev', float('nan')):.2e}  "
              f"gap {st.get('gap', float('nan')):.2e}  {time.time() - t:.1f}s", flush=True)
    sys.exit(1 if bad else 0)

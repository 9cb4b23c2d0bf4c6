"""Where does the recurrence's r differ from B - A w?  One GPU, single rank:
a three-step solve (restarts off), then w, kResid's rho (stored in x[0]'s
r-plane) and the recurrence's r of the same iterate (x[wpar], after the
replay launch) read back; rho = B - A w formed on the CPU (ops/torch_ref
assembly, fp64) checks kResid, and the gap rho - r is reported by node class
(interior / exterior / band) with its worst nodes.

    PROBE_GRID=2048x2048 PROBE_INIT=zero python tools/resid_probe.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import poisson_ellipse_openmp_mpi_cuda_amd as pe  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.ops import torch_ref  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402

nat = native()
for spec in os.environ.get("PROBE_GRID", "2048x2048").split(","):
    M, N = (int(v) for v in spec.split("x"))
    for init in os.environ.get("PROBE_INIT", "zero").split(","):
        prob = pe.EllipseProblem(M, N)
        opt = nat.SolveOptions()
        opt.init = nat.Init.Random if init == "random" else nat.Init.Zero
        opt.seed = 1234
        os.environ["PE_RESID_GAP"] = "1e300"  # (report only: no restart)
        s = nat.DeviceSolver(prob.to_native(), D.block(M, N, 1, 0), None, opt)
        res = s.solve()
        st = s.state()
        par = int(st["wpar"])
        fw = np.asarray(s.field(1))
        w = fw[1 : M + 2, 1 : N + 2].copy()  # field index 0 <-> local -1: global (i, j) at [i + 1, j + 1]
        rho_dev = np.asarray(s.field(0))[1 : M + 2, 1 : N + 2].copy()  # kResid stored rho in x[0]'s r-plane
        r = np.asarray(s.field(4))[1 : M + 2, 1 : N + 2].copy() if par == 1 else rho_dev * np.nan
        print(f"   solve: iters {res.iters} res_true {res.res_true:.4e} res_rec {res.res_rec:.4e} res_gap {res.res_gap:.4e}"
              f" b_norm {res.b_norm:.4e} fixj {st['fixj']}", flush=True)
        a, b, B = (t.numpy() for t in torch_ref.assemble(prob))
        import torch

        Aw = torch_ref.apply_A(torch.from_numpy(w), torch.from_numpy(a), torch.from_numpy(b), prob.h1, prob.h2).numpy()
        rho = B - Aw
        rho[0, :] = rho[-1, :] = rho[:, 0] = rho[:, -1] = 0.0
        r[0, :] = r[-1, :] = r[:, 0] = r[:, -1] = 0.0
        rho_dev[0, :] = rho_dev[-1, :] = rho_dev[:, 0] = rho_dev[:, -1] = 0.0
        dd = rho - rho_dev
        print(f"   kResid vs CPU rho: max |diff| {np.abs(dd).max():.3e}  |diff| {np.sqrt((dd**2).sum()):.3e}"
              f"  |rho| {np.sqrt((rho**2).sum()):.4e}", flush=True)
        if par != 1:
            print("   (wpar 0: the recurrence's r was overwritten by kResid's rho)")
            continue
        d = rho - r
        x = prob.A1 + np.arange(M + 1) * prob.h1
        y = prob.A2 + np.arange(N + 1) * prob.h2
        inside = (prob.cx * x[:, None] ** 2 + prob.cy * y[None, :] ** 2) < 1.0
        band = ~(np.isclose(a, 1.0) & np.isclose(b, 1.0)) & ~(np.isclose(a, 1 / prob.eps) & np.isclose(b, 1 / prob.eps))
        hh = prob.h1 * prob.h2
        nB = np.sqrt((B * B).sum())
        print(f"== {M}x{N} init {init}: iter {st['iter']} status {st['status']} wpar {par}  |B| {nB:.4e}"
              f"  |rho| {np.sqrt((rho**2).sum()):.4e}  |r| {np.sqrt((r**2).sum()):.4e}  |rho-r| {np.sqrt((d**2).sum()):.4e}"
              f"  (device res {[f'{v:.4e}' for v in st['res']]})", flush=True)
        for name, m in (("inside", inside & ~band), ("outside", ~inside & ~band), ("band", band)):
            m = m.copy()
            m[0, :] = m[-1, :] = m[:, 0] = m[:, -1] = False
            print(f"   {name:8s} nodes {m.sum():9d}  |rho-r| {np.sqrt((d[m] ** 2).sum()):.4e}  |r| {np.sqrt((r[m] ** 2).sum()):.4e}"
                  f"  max |w| {np.abs(w[m]).max() if m.any() else 0:.3e}")
        idx = np.argsort(np.abs(d).ravel())[-6:]
        for q in idx:
            i, j = divmod(int(q), N + 1)
            print(f"   worst ({i},{j}): rho {rho[i, j]: .4e} r {r[i, j]: .4e} w {w[i, j]: .4e} a {a[i, j]:.3e} b {b[i, j]:.3e}"
                  f" inside {bool(inside[i, j])}")
        # column / row profile of the gap
        cs = np.sqrt((d**2).sum(0))
        rs = np.sqrt((d**2).sum(1))
        print("   worst columns", [int(c) for c in np.argsort(cs)[-8:]], " worst rows", [int(c) for c in np.argsort(rs)[-8:]])
        del s

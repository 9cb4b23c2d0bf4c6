#!/usr/bin/env python3
"""Per-phase timeline of the LDS-resident sweep (resident.hip, PE_RES_STAMPS=1).

Every workgroup records s_memrealtime (100 MHz) at 8 points of each of the
first 64 iterations of a launch: 0 iteration start, 1 after phase A (p_k),
2 after phase B (s, r_k, z_k), 3 after the in-tile reduction, 4 after the
partial-sum stores drained, 5 after the grid barrier, 6 after the imports,
7 after the broadcast of the global sums.  Prints the median / max over
workgroups of every segment and the iteration period.

    PROBE_GRIDS="800x1200 40x40" python tools/res_stamp_probe.py
"""

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["PE_RES_STAMPS"] = "1"

from poisson_ellipse_openmp_mpi_cuda_amd import EllipseProblem, native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402

NAMES = ["A p_k", "B s,r,z", "C q + in-tile reduce", "store partials + drain", "grid barrier",
         "import ring + partials", "global sum broadcast", "-> next iteration"]


def probe(M, N, iters=64):
    nat = native()
    nat.set_device(0)
    prob = EllipseProblem(M, N)
    opt = nat.SolveOptions()
    opt.check_tol = False
    opt.chunk = iters
    s = nat.DeviceSolver(prob.to_native(), D.block(M, N, 1, 0), None, opt)
    if not s.resident:
        print(f"{M}x{N}: not resident")
        return
    s.reset()
    s.run_iterations(iters, False)
    s.synchronize()
    st = np.asarray(s.stamps(), dtype=np.int64).reshape(-1, 64, 8)[:, 8:iters, :]  # skip 8 warm iterations
    nwg = st.shape[0]
    seg = np.diff(st, axis=2) * 10e-3  # µs
    period = (st[:, 1:, 0] - st[:, :-1, 0]) * 10e-3
    print(f"== {M}x{N}: {nwg} workgroups, iterations 8..{iters - 1}")
    print(f"   period: median {np.median(period):7.2f} us  (max over wg of the mean {period.mean(axis=1).max():7.2f})")
    for j in range(7):
        x = seg[:, :, j]
        print(f"   {NAMES[j]:<26} median {np.median(x):6.2f}  p90 {np.percentile(x, 90):6.2f}  "
              f"max-wg-mean {x.mean(axis=1).max():6.2f} us")
    last = (st[:, 1:, 0] - st[:, :-1, 7]) * 10e-3
    print(f"   {NAMES[7]:<26} median {np.median(last):6.2f} us")
    # arrival skew at the barrier: spread of stamp 4 across workgroups per iteration
    arr = st[:, :, 4] * 10e-3
    print(f"   barrier arrival spread (max - min over wg): median {np.median(arr.max(0) - arr.min(0)):6.2f} us; "
          f"release spread {np.median((st[:, :, 5].max(0) - st[:, :, 5].min(0)) * 10e-3):6.2f} us")
    slow = np.argsort(-(st[:, :, 4] - st[:, :, 0]).mean(axis=1))[:5]
    print(f"   slowest workgroups to arrive: {slow.tolist()}")


def main():
    for g in os.environ.get("PROBE_GRIDS", "800x1200 40x40").split():
        M, N = (int(v) for v in g.split("x"))
        probe(M, N)


if __name__ == "__main__":
    main()

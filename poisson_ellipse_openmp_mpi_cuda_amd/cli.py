"""Command-line front end (Python).  Positional ``M N`` as in the reference
(``prog [M N]``, default 40 40: stage2-mpi/poisson_mpi_decomp.cpp:470-474).

    python -m poisson_ellipse_openmp_mpi_cuda_amd.cli 800 1200                    # 1 GPU
    python -m poisson_ellipse_openmp_mpi_cuda_amd.cli --backend omp --threads 8 400 600
    python -m poisson_ellipse_openmp_mpi_cuda_amd.cli --backend ranks --ranks 4 --threads 2 800 1200
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m poisson_ellipse_openmp_mpi_cuda_amd.cli 8192 8192
    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 -m poisson_ellipse_openmp_mpi_cuda_amd.cli --backend dist-cpu 400 600

Prints the reference's result lines (``--legacy``, default) and/or a JSON
report (``--json``), the L2/max error against the analytic solution, and
optionally dumps w (``--dump w.npy``, plus ``--pgm w.pgm``).
"""

from __future__ import annotations

import argparse
import os
import sys

from .models.ellipse import PRESETS, EllipseProblem
from .solver import BACKENDS, solve
from .utils import dump as _dump
from .utils.report import json_report, legacy_lines


def build_parser():
    ap = argparse.ArgumentParser(prog="pe", description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("M", nargs="?", type=int, default=None)
    ap.add_argument("N", nargs="?", type=int, default=None)
    ap.add_argument("--preset", choices=sorted(PRESETS), default=None)
    ap.add_argument("--backend", choices=BACKENDS, default=os.environ.get("PE_BACKEND", "hip"))
    ap.add_argument("--ranks", type=int, default=1, help="thread-ranks (ranks) or virtual ranks (hip-group)")
    ap.add_argument("--threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "1") or 1))
    ap.add_argument("--decomp", default=None,
                    help="aspect | reference | rows | cols | device | <Px>x<Py> (e.g. 4x2); "
                         "default: device for the GPU backends, aspect otherwise")
    ap.add_argument("--init", choices=("zero", "random"), default="zero")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--tol", type=float, default=1e-6)
    ap.add_argument("--max-iter", type=int, default=-1)
    ap.add_argument("--norm", choices=("weighted", "unweighted"), default="weighted")
    ap.add_argument("--variant", type=int, default=0, help="device arithmetic: 0 fast (default), 1 reference-exact")
    ap.add_argument("--algo", choices=("auto", "classic", "fused", "two-step", "three-step"), default="auto",
                    help="device iteration: fused single-sweep (1 kernel, 1 reduction), two-step / three-step (2 / 3 "
                         "iterations per sweep, 1 reduction per sweep) or classic (2 + 2)")
    ap.add_argument("--timing", action="store_true", help="per-phase device event timers")
    ap.add_argument("--checkpoint", default=None, help="hip: checkpoint file prefix (one file per rank: PREFIX.r<rank>)")
    ap.add_argument("--checkpoint-every", type=int, default=0, help="hip: iterations between checkpoints")
    ap.add_argument("--resume", default=None, help="hip: resume from checkpoint prefix")
    ap.add_argument("--log-every", type=int, default=0, help="print ||dw|| every K iterations (hip: chunk-granular)")
    ap.add_argument("--no-graph", action="store_true", help="(default) eager launches")
    ap.add_argument("--graph", action="store_true", help="replay chunks of iterations from hipGraphs")
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--quiet", action="store_true", help="suppress the legacy lines")
    ap.add_argument("--dump", default=None, help="write w (interior) to this .npy")
    ap.add_argument("--pgm", default=None, help="write a grey-scale image of w")
    return ap


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    prob = PRESETS[a.preset] if a.preset else EllipseProblem()
    if a.M is not None and a.N is not None:
        prob = prob.with_grid(a.M, a.N)
    prob.tol = a.tol
    prob.max_iter = a.max_iter
    prob.norm = a.norm
    want_w = bool(a.dump or a.pgm)
    rep = solve(prob, backend=a.backend, ranks=a.ranks, threads=a.threads, decomp=a.decomp, init=a.init,
                seed=a.seed, return_w=want_w, variant=a.variant, timing=a.timing, graph=a.graph and not a.no_graph,
                algo=a.algo, checkpoint=a.checkpoint, checkpoint_every=a.checkpoint_every, resume=a.resume,
                log_every=a.log_every)
    if rep.rank != 0:
        return 0
    if not a.quiet:
        print(legacy_lines(rep, a.tol))
        print(f"   Process grid {rep.Px}x{rep.Py} | iters/s ~ {rep.iters_per_s:.1f} | L2 error in D ~ {rep.l2_err:.6e}"
              f" | max error in D ~ {rep.max_err:.6e}")
    if a.json:
        print(json_report(rep))
    if want_w and rep.w is not None:
        if a.dump:
            _dump.save(a.dump, rep.w, prob, rep)
        if a.pgm:
            _dump.write_pgm(a.pgm, rep.w)
    sys.stdout.flush()
    if rep.nonfinite:
        print("error: a reduced scalar became NaN/Inf; solve stopped", file=sys.stderr)
        return 3
    return 0


if __name__ == "__main__":
    sys.exit(main())

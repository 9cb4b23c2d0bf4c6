"""Multi-process CPU ranks over torch.distributed (gloo): the MPI stage2/3
pattern (halo Isend/Irecv + scalar Allreduce, poisson_mpi_decomp.cpp:241-460)
on the framework's callback transport.  Iteration counts and the gathered
solution must equal the single-process oracle."""

import os
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, M, N, decomp, threads, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from poisson_ellipse_openmp_mpi_cuda_amd import EllipseProblem, solve

    rep = solve(EllipseProblem(M, N), backend="dist-cpu", decomp=decomp, threads=threads, return_w=True)
    if rank == 0:
        out.put((rep.iters, rep.converged, rep.Px, rep.Py, rep.l2_err, rep.w))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,decomp,threads", [(2, "aspect", 1), (3, "reference", 1), (4, "aspect", 2)])
def test_gloo_ranks_match_serial(world, decomp, threads):
    from poisson_ellipse_openmp_mpi_cuda_amd import EllipseProblem, solve

    M, N = 90, 70
    ref = solve(EllipseProblem(M, N), backend="serial", return_w=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, M, N, decomp, threads, q)) for r in range(world)]
    for p in procs:
        p.start()
    iters, conv, Px, Py, l2, w = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert conv and iters == ref.iters
    assert Px * Py == world
    np.testing.assert_allclose(w, ref.w, rtol=0, atol=1e-12)
    assert l2 == pytest.approx(ref.l2_err, rel=1e-9)

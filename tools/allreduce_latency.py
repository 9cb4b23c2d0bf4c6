"""Latency of the per-iteration 7-double sum through the device transports.

    torchrun --nproc-per-node N tools/allreduce_latency.py   (PE_COMM / PE_ALLREDUCE as for the solver)

On a multi-GPU node the default transport is RCCL; PE_ALLREDUCE=p2p wraps it
with the one-shot IPC/xGMI kernel.  On a one-GPU box run it with
PE_COMM=host (several ranks on the one GPU): only the P2P path is then on
the device (the host-staged sum is a host round trip)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from poisson_ellipse_openmp_mpi_cuda_amd.parallel import dist as D  # noqa: E402

ctx = D.init()
comm = D.rccl_comm(ctx)
iters = int(os.environ.get("ITERS", "2000"))
us = comm.bench_allreduce(7, iters) if comm is not None else 0.0
if ctx.rank == 0:
    print(json.dumps({"comm": comm.name if comm else "self", "ranks": ctx.world, "n": 7, "iters": iters,
                      "us_per_allreduce": round(us, 3)}), flush=True)

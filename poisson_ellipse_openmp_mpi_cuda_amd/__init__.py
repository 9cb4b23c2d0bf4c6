"""MI355X-native 2D Poisson / fictitious-domain PCG framework.

Capabilities of ``mxy-kit/poisson-ellipse-openmp-mpi-cuda`` (sequential,
OpenMP, MPI, MPI+OpenMP and MPI+CUDA Jacobi-PCG solvers for -Δu = 1 on the
ellipse x² + 4y² < 1 embedded in [-1,1]×[-0.6,0.6]) rebuilt MI355X-first:

* native C++ core (``csrc/``): decomposition, CPU backends (serial / OpenMP /
  thread-ranks = the reference's stage0..3), device runtime;
* hand-written gfx950 HIP kernels (``csrc/hip/kernels.hip``): fused
  direction-update+stencil+dots and fused update+stencil+preconditioner+dot
  marching kernels with on-the-fly fictitious-domain coefficients;
* RCCL over xGMI for the 2D domain decomposition (one process per GPU,
  bootstrapped through ``torch.distributed``);
* a PyTorch fp64 oracle (``ops.torch_ref``) used by the tests.

Subpackages: ``models`` (problem definitions), ``ops`` (kernels / oracle),
``parallel`` (decomposition, torch.distributed bootstrap, transports),
``utils`` (reporting, timers, dumps).
"""

from .models.ellipse import EllipseProblem, REFERENCE_PROBLEM  # noqa: F401
from .solver import solve, SolveReport  # noqa: F401
from ._loader import native, native_available  # noqa: F401

__version__ = "0.1.0"

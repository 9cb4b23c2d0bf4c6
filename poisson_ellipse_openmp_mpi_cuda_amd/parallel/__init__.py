"""Parallelism: 2D domain decomposition and the transports (torch.distributed
bootstrap, native RCCL over xGMI for GPU ranks, gloo callbacks for CPU
ranks, thread ranks and virtual ranks inside the native core)."""

from . import decomp  # noqa: F401

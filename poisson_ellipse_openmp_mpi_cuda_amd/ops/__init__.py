"""Operators: the PyTorch fp64 oracle (``torch_ref``) and thin wrappers around
the native gfx950 kernels (``device``)."""

from . import torch_ref  # noqa: F401

"""Problem definitions (the "model family" of this framework)."""

from .ellipse import EllipseProblem, REFERENCE_PROBLEM, PRESETS, GOLDEN_ITERS, GOLDEN_L2  # noqa: F401

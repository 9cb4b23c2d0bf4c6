"""Utilities: reporting (legacy lines / JSON), solution dumps and timers."""

from . import report  # noqa: F401

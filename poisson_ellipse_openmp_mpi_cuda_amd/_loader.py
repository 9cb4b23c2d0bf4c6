"""Loader for the in-tree native extension ``_native`` (C++/HIP/RCCL).

The extension is built in-tree by ``make`` (or ``__graft_entry__.build()``).
PyTorch is imported first on purpose: the extension links
``libamdhip64.so.7`` / ``librccl.so.1``, and with torch already loaded the
dynamic linker binds them to torch's copies (same SONAME), so torch and the
framework share ONE HIP runtime and one RCCL in the process.

On a GPU box a missing or stale extension is a hard error (no silent
fallback to a PyTorch path): set ``PE_ALLOW_NO_NATIVE=1`` only for docs
builds.
"""

from __future__ import annotations

import importlib
import os

_NATIVE = None
_ERR: Exception | None = None


def _load():
    global _NATIVE, _ERR
    if _NATIVE is not None or _ERR is not None:
        return
    try:
        import torch  # noqa: F401  (bind HIP/RCCL to torch's copies first)
    except Exception:  # pragma: no cover - torch is part of the image
        pass
    try:
        _NATIVE = importlib.import_module(__package__ + "._native")
    except Exception as e:  # pragma: no cover - exercised when unbuilt
        _ERR = e


def native_available() -> bool:
    _load()
    return _NATIVE is not None


def native():
    """Return the native module or raise a loud, actionable error."""
    _load()
    if _NATIVE is None:
        raise RuntimeError(
            "poisson_ellipse native extension is not built or failed to load "
            f"({_ERR!r}); run `make -j8` (or python -c 'import __graft_entry__ as g; g.build()') "
            "in the repository root"
        )
    return _NATIVE


def gpu_available() -> bool:
    """True when a HIP device is visible to the native runtime."""
    if os.environ.get("PE_FORCE_CPU"):
        return False
    try:
        return native().device_count() > 0
    except Exception:
        return False

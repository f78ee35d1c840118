"""Loader for the in-tree native extension ``mobilefinetuner_amd/_C.so``.

GPU code paths call :func:`native` and FAIL LOUDLY when the extension is missing — there is no
eager fallback.  The op layer has no host path of its own: host tensors are served only when the
test-suite's fp32 oracle (``tests/oracle``) is installed, and raise otherwise.
"""
from __future__ import annotations

import os

_C = None
_ERR = None


def native():
    """Return the compiled extension module, building it on first use if needed."""
    global _C, _ERR
    if _C is not None:
        return _C
    try:
        import torch  # noqa: F401  (the extension links against torch's HIP runtime)
        from . import _C as mod  # type: ignore
    except ImportError as e:  # not built yet -> build in-tree once
        if os.environ.get("MFT_NO_AUTOBUILD"):
            raise RuntimeError(f"mobilefinetuner_amd native extension not available: {e}") from e
        from ._build import build
        build()
        from . import _C as mod  # type: ignore
    _C = mod
    return _C


def available() -> bool:
    try:
        native()
        return True
    except Exception:  # pragma: no cover
        return False

"""Loader for the in-tree native core (``_mdfx`` + ``lib/libmdfx.so``).

torch must be imported before the native module: torch ships its own ``libamdhip64.so.7`` and
``librccl.so.1``; loading torch first makes the native core bind to those same instances (one HIP
runtime per process). The module fails loudly if the extension was not built (``make -j8``) —
there is no silent pure-Python fallback for the compute path.
"""

from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  (must precede the native import, see module docstring)

_mod = None


def native():
    """Return the ``_mdfx`` extension module, importing it on first use."""
    global _mod
    if _mod is None:
        try:
            _mod = importlib.import_module("mpi_cuda_process_amd._mdfx")
        except ImportError as e:  # pragma: no cover - exercised only when unbuilt
            root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
            raise ImportError(
                "mdfx native core is not built: run `make -j8` in %s (or "
                "`python -c 'import __graft_entry__ as g; g.build()'`). Original error: %s" % (root, e)
            ) from e
    return _mod


def native_library_path() -> str:
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libmdfx.so")


def hip_available() -> bool:
    """True when a HIP device is usable from this process."""
    return torch.cuda.is_available() and native().hip_device_count() > 0


def require_hip() -> None:
    if not hip_available():
        raise RuntimeError("no HIP device available (this path needs an MI355X / gfx950 GPU)")

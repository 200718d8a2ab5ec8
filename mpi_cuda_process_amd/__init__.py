"""mpi_cuda_process_amd (mdfx): an MI355X-native multi-GPU finite-difference stencil engine.

Capabilities of Rodrigovicente/MPI-CUDA-Process (2D 5-point MDF heat/Jacobi and Game of Life,
slab-decomposed across ranks with ghost-row exchange and interior/boundary stream overlap),
re-designed for AMD Instinct MI355X (gfx950): hand-written CDNA4 HIP kernels (2.5D z-marching,
wave64, DPP lane shifts + LDS seams, XCD-aware tiling, fused multi-step temporal blocking), a
native C++ engine with two HIP streams per slab and double buffering, and RCCL point-to-point
halo exchange over xGMI — plus 3D 7-point and 27-point stencils, fp64, residuals,
checkpoint/resume and hipGraph replay.

Entry points: :class:`Simulation` (decomposed, multi-slab / multi-GPU runs), :func:`advance`
(functional: k steps of a dense grid tensor), ``python -m mpi_cuda_process_amd`` (CLI).

Layout::

    models/    problem families (mdf2d, life2d, heat3d, box27)
    ops/       torch-facing kernel ops + plain-PyTorch reference stencils
    parallel/  slab decomposition, torch.distributed bootstrap, torch p2p transport
    utils/     metrics, ASCII output, CLI helpers
    engine.py  Simulation (native mdfx::Solver)
    lib/       libmdfx.so (native core: kernels, runtime, transports, engine)
"""

import os as _os

import sys as _sys
import warnings as _warnings

# hipGraph replay on ONE hardware queue. The HIP runtime's graph executor spreads a captured
# cycle's parallel branches (interior sweep || boundary sweep + halo exchange) over several internal
# queues, and the cross-queue dependencies made replayed cycles 1.4-2x slower than the same work
# launched eagerly (bench/graph_probe.py, profiles/r04_session_c/); on one queue they replay close
# to eager. Side effect: the runtime reads the variable once, when it starts, and applies it to EVERY
# hipGraph of the process, the application's own torch CUDA graphs included. It is only set when
# unset (a caller's value wins), and it cannot take effect if HIP started before this import:
# GRAPH_QUEUES records which case holds (also in Simulation.options) and a warning says so.
_torch = _sys.modules.get("torch")
_hip_started = bool(_torch is not None and getattr(_torch, "cuda", None) is not None and
                    _torch.cuda.is_initialized())
if "DEBUG_HIP_FORCE_GRAPH_QUEUES" in _os.environ:
    GRAPH_QUEUES = "caller's DEBUG_HIP_FORCE_GRAPH_QUEUES=%s" % _os.environ["DEBUG_HIP_FORCE_GRAPH_QUEUES"]
elif _hip_started:
    GRAPH_QUEUES = "runtime default (HIP was initialised before this import)"
    _warnings.warn("mpi_cuda_process_amd was imported after HIP started, so DEBUG_HIP_FORCE_GRAPH_QUEUES=1 "
                   "cannot take effect: replayed hipGraph cycles run on several hardware queues (slower than "
                   "eager steps, and not the schedule measured). Import the package, or set the variable, "
                   "before the first GPU call.", RuntimeWarning, stacklevel=2)
else:
    _os.environ["DEBUG_HIP_FORCE_GRAPH_QUEUES"] = "1"
    GRAPH_QUEUES = "one queue (DEBUG_HIP_FORCE_GRAPH_QUEUES=1 set by mpi_cuda_process_amd)"

from ._native import hip_available, native, require_hip  # noqa: F401,E402  (imports torch first)
from .engine import Simulation  # noqa: F401
from .models import InitCondition, Problem, box27, from_name, heat3d, life2d, mdf2d  # noqa: F401
from .ops import advance  # noqa: F401

__version__ = "0.1.0"

__all__ = ["Simulation", "Problem", "InitCondition", "mdf2d", "life2d", "heat3d", "box27", "from_name",
           "advance", "native", "hip_available", "require_hip"]

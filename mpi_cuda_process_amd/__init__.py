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

# hipGraph replay on ONE hardware queue. The HIP runtime's graph executor spreads a captured
# cycle's parallel branches (interior sweep || boundary sweep + halo exchange) over several internal
# queues, and the cross-queue dependencies made replayed cycles 1.4-2x slower than the same work
# launched eagerly (bench/graph_probe.py, profiles/r04_session_c/); on one queue replay matches
# eager. Read when the runtime starts, so it must be set before the first HIP call of the process.
_os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "1")

from ._native import hip_available, native, require_hip  # noqa: F401,E402  (imports torch first)
from .engine import Simulation  # noqa: F401
from .models import InitCondition, Problem, box27, from_name, heat3d, life2d, mdf2d  # noqa: F401
from .ops import advance  # noqa: F401

__version__ = "0.1.0"

__all__ = ["Simulation", "Problem", "InitCondition", "mdf2d", "life2d", "heat3d", "box27", "from_name",
           "advance", "native", "hip_available", "require_hip"]

"""Helpers around the engine: metrics, the reference's ASCII output, checkpoint/dump files.

* :func:`gcells`, :func:`hbm_roof_gcells`, :func:`metrics_record` — the numbers every bench and
  CLI reports (GCells/s = cells x time steps / s, per-GPU share, effective HBM bytes/s).
* :func:`format_array` / :func:`print_array` — the reference's ``print_array``
  (``kernel.cu:115-129``): '0' for a cell equal to 1, ' ' otherwise, blank lines around.
* :func:`read_checkpoint` — reassemble a checkpoint / ``--dump`` directory (per-slab raw + JSON
  header, written by ``mdfx::Solver::save_checkpoint``) into one dense numpy grid.
"""

from .ascii import format_array, print_array  # noqa: F401
from .checkpoint import read_checkpoint  # noqa: F401
from .metrics import bytes_per_cell_per_step, gcells, hbm_roof_gcells, metrics_record  # noqa: F401

__all__ = ["format_array", "print_array", "read_checkpoint", "gcells", "hbm_roof_gcells", "metrics_record",
           "bytes_per_cell_per_step"]

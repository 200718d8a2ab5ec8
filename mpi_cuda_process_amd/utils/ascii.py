"""The reference's ASCII grid dump (``print_array``, kernel.cu:115-129 / MDF_kernel.cu:72-86)."""

from __future__ import annotations

import sys

import numpy as np


def _rows(a: np.ndarray) -> str:
    return "\n" + "".join("".join("0" if v == 1 else " " for v in row) + "\n" for row in a) + "\n"


def format_array(grid: np.ndarray) -> str:
    """'0' for a cell equal to 1, ' ' otherwise, a newline per row, a blank line before and after.

    2D grids (``(h, w)`` or ``(h, 1, w)``) print as one block, like the reference; 3D grids
    ``(nz, ny, nx)`` print plane by plane after a ``z=<k>`` label (the native CLI's format)."""
    g = np.asarray(grid)
    if g.ndim == 3 and g.shape[1] > 1:
        return "".join("z=%d" % z + _rows(g[z]) for z in range(g.shape[0]))
    return _rows(g.reshape(-1, g.shape[-1]))


def print_array(grid: np.ndarray, out=None) -> None:
    (out or sys.stdout).write(format_array(grid))

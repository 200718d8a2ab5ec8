"""Slab decomposition math (mirrors ``mdfx::SlabDecomposition`` in csrc/core/common.cpp).

The first ``nz % parts`` slabs get one extra plane. Reference: MDF_kernel.cu:30,54 split at
exactly ``size/2`` between two hard-coded ranks; this works for any 1 <= P <= nz.
"""

from __future__ import annotations

from typing import List, Tuple


def slab_bounds(nz: int, parts: int) -> List[Tuple[int, int]]:
    if parts < 1:
        raise ValueError("need at least one part")
    if nz < parts:
        raise ValueError("cannot split %d planes over %d ranks" % (nz, parts))
    base, rem = divmod(nz, parts)
    out, z = [], 0
    for p in range(parts):
        n = base + (1 if p < rem else 0)
        out.append((z, z + n))
        z += n
    return out


def owner(gz: int, nz: int, parts: int) -> int:
    if not 0 <= gz < nz:
        raise ValueError("plane outside the grid")
    base, rem = divmod(nz, parts)
    split = rem * (base + 1)
    if gz < split:
        return gz // (base + 1)
    return rem + (gz - split) // base


def neighbors(rank: int, parts: int) -> Tuple[int, int]:
    """(lower, upper) neighbour slab of ``rank``; -1 at the global boundary."""
    return (rank - 1 if rank > 0 else -1, rank + 1 if rank + 1 < parts else -1)


def pencil_bounds(nz: int, ny: int, pz: int, py: int) -> List[Tuple[Tuple[int, int], Tuple[int, int]]]:
    """((z0, z1), (y0, y1)) of every rank of a pz x py (z, y) pencil decomposition (mirrors
    ``mdfx::PencilDecomposition``): rank r = rz * py + ry; its z neighbours are r -/+ py, its y
    neighbours r -/+ 1."""
    zs, ys = slab_bounds(nz, pz), slab_bounds(ny, py)
    return [(zs[r // py], ys[r % py]) for r in range(pz * py)]


def pencil_neighbors(rank: int, pz: int, py: int) -> Tuple[int, int, int, int]:
    """(z-lower, z-upper, y-lower, y-upper) neighbour of ``rank``; -1 at the global boundary."""
    rz, ry = divmod(rank, py)
    return (rank - py if rz > 0 else -1, rank + py if rz + 1 < pz else -1,
            rank - 1 if ry > 0 else -1, rank + 1 if ry + 1 < py else -1)

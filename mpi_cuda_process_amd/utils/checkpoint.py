"""Checkpoint / dump files: one raw little-endian slab per rank plus a JSON header
(``slab_<r>.bin`` / ``slab_<r>.json``, format ``mdfx-slab-v1``), in global plane order so any
decomposition can be reassembled (csrc/engine/solver.cpp save_checkpoint)."""

from __future__ import annotations

import json
import os
from typing import List, Tuple

import numpy as np

_DT = {"f32": np.float32, "f64": np.float64, "u8": np.uint8}


def read_checkpoint(path: str) -> Tuple[np.ndarray, List[dict]]:
    """The dense global grid ``(nz, ny, nx)`` and the per-slab headers of a checkpoint directory.

    Only raw bytes and JSON are read (nothing is unpickled)."""
    metas = []
    for f in sorted(os.listdir(path)):
        if f.startswith("slab_") and f.endswith(".json"):
            with open(os.path.join(path, f)) as fh:
                metas.append(json.load(fh))
    if not metas:
        raise FileNotFoundError("no slab_<r>.json headers in %s" % path)
    m0 = metas[0]
    if any(m.get("format") != "mdfx-slab-v1" for m in metas):
        raise ValueError("not an mdfx-slab-v1 checkpoint")
    dt = _DT[m0["dtype"]]
    grid = np.zeros((m0["nz"], m0["ny"], m0["nx"]), dtype=dt)
    covered = np.zeros(m0["nz"], dtype=bool)
    for m in metas:
        n = (m["z1"] - m["z0"]) * m["ny"] * m["nx"]
        raw = np.fromfile(os.path.join(path, "slab_%d.bin" % m["rank"]), dtype=dt)
        if raw.size != n:
            raise ValueError("slab %d: %d values, expected %d" % (m["rank"], raw.size, n))
        grid[m["z0"]:m["z1"]] = raw.reshape(m["z1"] - m["z0"], m["ny"], m["nx"])
        covered[m["z0"]:m["z1"]] = True
    if not covered.all():
        raise ValueError("the slabs do not cover every plane")
    return grid, metas

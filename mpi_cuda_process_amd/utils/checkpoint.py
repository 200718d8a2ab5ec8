"""Checkpoint / dump files: one raw little-endian slab per rank plus a JSON header
(``slab_<r>.bin`` / ``slab_<r>.json``, format ``mdfx-slab-v1``; a pencil's header adds its rows
``y0``, ``y1``), in global plane order so any decomposition can be reassembled
(csrc/engine/solver.cpp save_checkpoint)."""

from __future__ import annotations

import json
import os
from typing import List, Tuple

import numpy as np

_DT = {"f32": np.float32, "f64": np.float64, "u8": np.uint8}


def read_checkpoint(path: str) -> Tuple[np.ndarray, List[dict]]:
    """The dense global grid ``(nz, ny, nx)`` and the per-slab headers of a checkpoint directory.

    Only raw bytes and JSON are read (nothing is unpickled)."""
    def header(r):
        f = os.path.join(path, "slab_%d.json" % r)
        if not os.path.exists(f):
            raise ValueError("checkpoint %s is incomplete: slab_%d.json is missing" % (path, r))
        with open(f) as fh:
            return json.load(fh)

    if not os.path.exists(os.path.join(path, "slab_0.json")):
        raise FileNotFoundError("no slab_0.json header in %s" % path)
    m0 = header(0)
    # slab_0 names the writer's rank count; files of an older save with more ranks are ignored
    metas = [m0] + [header(r) for r in range(1, int(m0["nranks"]))]
    if any(m.get("format") != "mdfx-slab-v1" for m in metas):
        raise ValueError("not an mdfx-slab-v1 checkpoint")
    for m in metas:
        if m["nranks"] != m0["nranks"] or m["step"] != m0["step"]:
            raise ValueError("slab %d (nranks %d, step %d) does not match slab_0 (nranks %d, step %d)"
                             % (m["rank"], m["nranks"], m["step"], m0["nranks"], m0["step"]))
    dt = _DT[m0["dtype"]]
    grid = np.zeros((m0["nz"], m0["ny"], m0["nx"]), dtype=dt)
    covered = np.zeros((m0["nz"], m0["ny"]), dtype=bool)
    for m in metas:
        # slabs own every row; a (z, y) pencil's header also names its rows [y0, y1)
        y0, y1 = m.get("y0", 0), m.get("y1", m["ny"])
        shape = (m["z1"] - m["z0"], y1 - y0, m["nx"])
        raw = np.fromfile(os.path.join(path, "slab_%d.bin" % m["rank"]), dtype=dt)
        if raw.size != shape[0] * shape[1] * shape[2]:
            raise ValueError("slab %d: %d values, expected %d" % (m["rank"], raw.size, shape[0] * shape[1] * shape[2]))
        grid[m["z0"]:m["z1"], y0:y1] = raw.reshape(shape)
        covered[m["z0"]:m["z1"], y0:y1] = True
    if not covered.all():
        raise ValueError("the slabs do not cover every plane")
    return grid, metas

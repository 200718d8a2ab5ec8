"""Throughput metrics shared by bench.py and the CLIs."""

from __future__ import annotations

from typing import Optional

# float4 streaming copy on one MI355X (MI355X_MICROARCH.md); the 8.0 TB/s spec is not reachable
HBM_MEASURED_TBPS = 6.29
_ESIZE = {"f32": 4, "f64": 8, "u8": 1}


def gcells(cells: int, steps: int, seconds: float) -> float:
    """GCells/s: grid cells x time steps per second / 1e9 (every step updates every cell)."""
    return cells * steps / seconds / 1e9 if seconds > 0 else 0.0


def bytes_per_cell_per_step(dtype: str) -> int:
    """HBM bytes of an ideal single sweep: one read and one write of the field."""
    return 2 * _ESIZE[dtype]


def hbm_roof_gcells(dtype: str, n_gpus: int = 1, tbps: float = HBM_MEASURED_TBPS) -> float:
    """GCells/s of one single-step sweep per time step at the copy roof (fused sweeps exceed it)."""
    return tbps * 1e12 / bytes_per_cell_per_step(dtype) / 1e9 * n_gpus


def metrics_record(problem, steps: int, seconds: float, n_gpus: int, extra: Optional[dict] = None) -> dict:
    """The JSON fields every mdfx front end reports for a timed run."""
    v = gcells(problem.cells, steps, seconds)
    rec = {"metric": "GCells/s", "value": round(v, 4), "unit": "GCells/s", "stencil": problem.kind,
           "dtype": problem.dtype, "grid": [problem.nx, problem.ny, problem.nz], "steps": steps,
           "seconds": round(seconds, 6), "ms_per_step": round(seconds / max(steps, 1) * 1e3, 4), "n_gpus": n_gpus,
           "gcells_per_gpu": round(v / max(n_gpus, 1), 4)}
    if extra:
        rec.update(extra)
    return rec

"""Torch-facing kernel ops: engine-layout field tensors and single region updates.

A *field* is a torch tensor in the engine's storage layout for one slab: shape
``(planes, ny, pitch)`` with ``planes = (z1 - z0) + 2 * halo`` (ghost planes included) and rows
padded to 256 B (``pitch >= nx``). :func:`apply_stencil` runs the native kernel (the hand-written
gfx950 kernel on a HIP tensor, the CPU oracle on a CPU tensor) for storage planes
``[lz_begin, lz_end)`` on the current torch stream.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from .._native import native
from ..models import Problem
from . import reference  # noqa: F401

TORCH_DTYPE = {"f32": torch.float32, "f64": torch.float64, "u8": torch.uint8}


@dataclass
class FieldLayout:
    nx: int
    ny: int
    nz: int
    z0: int
    z1: int
    halo: int
    dtype: str
    pitch: int
    plane: int
    planes: int
    nbytes: int

    @classmethod
    def make(cls, problem: Problem, z0: int = 0, z1: Optional[int] = None, halo: int = 1) -> "FieldLayout":
        z1 = problem.nz if z1 is None else z1
        d = native().layout(problem.nx, problem.ny, problem.nz, z0, z1, halo, problem.dtype)
        return cls(d["nx"], d["ny"], d["nz"], d["z0"], d["z1"], d["halo"], problem.dtype, d["pitch"],
                   d["plane"], d["planes"], d["bytes"])

    @property
    def owned(self) -> slice:
        return slice(self.halo, self.halo + self.z1 - self.z0)


def alloc_field(layout: FieldLayout, device="cpu") -> torch.Tensor:
    """Zeroed storage for one slab, including the allocation slack the vector kernels rely on."""
    dt = TORCH_DTYPE[layout.dtype]
    es = torch.empty((), dtype=dt).element_size()
    flat = torch.zeros((layout.nbytes + es - 1) // es, dtype=dt, device=device)
    return flat[: layout.planes * layout.plane].view(layout.planes, layout.ny, layout.pitch)


def _device_index(t: torch.Tensor) -> int:
    return -1 if t.device.type == "cpu" else (t.device.index if t.device.index is not None else torch.cuda.current_device())


def _check(t: torch.Tensor, layout: FieldLayout):
    if t.dtype != TORCH_DTYPE[layout.dtype]:
        raise TypeError("field dtype %s does not match layout %s" % (t.dtype, layout.dtype))
    if tuple(t.shape) != (layout.planes, layout.ny, layout.pitch) or not t.is_contiguous():
        raise ValueError("field must be a contiguous (planes, ny, pitch) = %s tensor" %
                         ((layout.planes, layout.ny, layout.pitch),))


def init_field(problem: Problem, layout: FieldLayout, t: torch.Tensor, init=None) -> torch.Tensor:
    """Fill a field (ghost planes too) with the problem's initial condition from global indices."""
    _check(t, layout)
    ic = init or problem.init
    dev = _device_index(t)
    stream = torch.cuda.current_stream(t.device).cuda_stream if dev >= 0 else 0
    native().init_field(ic.kind if ic.kind != "compat" else "life", layout.dtype, t.data_ptr(), layout.nx,
                        layout.ny, layout.nz, layout.z0, layout.z1, layout.halo, dev, stream, seed=ic.seed,
                        lo=ic.lo, hi=ic.hi, value=ic.value, edge=ic.edge, interior=ic.interior,
                        density=ic.density)
    return t


def apply_stencil(problem: Problem, layout: FieldLayout, src: torch.Tensor, dst: torch.Tensor,
                  lz_begin: Optional[int] = None, lz_end: Optional[int] = None,
                  resid: Optional[torch.Tensor] = None, steps: int = 1,
                  second: Optional[tuple] = None) -> None:
    """One update of storage planes [lz_begin, lz_end) (default: all owned planes) src -> dst.

    ``resid`` (float64 scalar tensor on the same device), when given, accumulates
    sum((dst - src)^2) over the region. ``steps`` > 1 fuses that many time steps into one sweep
    (temporal blocking; needs ``layout.halo >= steps`` and valid ghosts that deep); the residual
    then covers the last step. ``second`` = (lz_begin, lz_end) of a second region updated by the
    same call (the engine's pair of boundary regions; one launch for the fused 3D 7-point sweep).
    """
    _check(src, layout)
    _check(dst, layout)
    if src.device != dst.device:
        raise ValueError("src and dst must be on the same device")
    lb = layout.halo if lz_begin is None else lz_begin
    le = layout.halo + layout.z1 - layout.z0 if lz_end is None else lz_end
    if not (layout.halo <= lb <= le <= layout.halo + layout.z1 - layout.z0):
        raise ValueError("region must lie inside the owned planes")
    rp = 0
    if resid is not None:
        if resid.dtype != torch.float64 or resid.device != src.device or resid.numel() != 1:
            raise ValueError("resid must be a float64 scalar on the field's device")
        rp = resid.data_ptr()
    dev = _device_index(src)
    stream = torch.cuda.current_stream(src.device).cuda_stream if dev >= 0 else 0
    native().stencil(problem.kind, layout.dtype, src.data_ptr(), dst.data_ptr(), layout.nx, layout.ny,
                     layout.nz, layout.z0, layout.z1, layout.halo, lb, le, dev, stream, rp,
                     steps=steps, lz2_begin=second[0] if second else 0, lz2_end=second[1] if second else 0,
                     **problem.coef_kwargs())


def dense_to_field(problem: Problem, dense: torch.Tensor, layout: FieldLayout, t: torch.Tensor):
    """Copy a dense global grid (nz, ny, nx) into a field's owned + available ghost planes."""
    lo = max(layout.z0 - layout.halo, 0)
    hi = min(layout.z1 + layout.halo, layout.nz)
    for gz in range(lo, hi):
        t[gz - layout.z0 + layout.halo, :, : layout.nx] = dense[gz]
    return t


def field_to_dense(layout: FieldLayout, t: torch.Tensor) -> torch.Tensor:
    """The owned planes of a field as a dense (z1-z0, ny, nx) tensor."""
    return t[layout.owned, :, : layout.nx].contiguous()


def set_kernel_variant(name: str) -> None:
    """Select the HIP kernel family: "auto"/"tuned" (2.5D z-march kernels) or "naive"."""
    native().set_kernel_variant(name)


def kernel_variant() -> str:
    return native().kernel_variant()


__all__ = ["FieldLayout", "alloc_field", "init_field", "apply_stencil", "dense_to_field", "field_to_dense",
           "set_kernel_variant", "kernel_variant", "reference", "TORCH_DTYPE"]


def advance(problem: Problem, grid: torch.Tensor, steps: int, temporal: int = 0) -> torch.Tensor:
    """Functional API: ``steps`` time steps of ``problem``'s stencil applied to a dense global grid
    ``(nz, ny, nx)`` (2D problems: ``(h, 1, w)`` or ``(h, w)``), on the grid's device (HIP kernels
    on a GPU tensor, the CPU oracle otherwise). Returns a new dense tensor; the input is untouched.

    ``temporal`` fuses that many steps per sweep (0 = the deepest fused kernel that exists for the
    problem on this device, as the CLI's auto mode). The result is bitwise identical for every depth.
    """
    squeeze = grid.dim() == 2
    g = grid.unsqueeze(1) if squeeze else grid
    if tuple(g.shape) != (problem.nz, problem.ny, problem.nx):
        raise ValueError("grid shape %s does not match the problem (%d, %d, %d)" %
                         (tuple(grid.shape), problem.nz, problem.ny, problem.nx))
    dev = g.device
    if temporal <= 0:
        want = native().hip_fused_depth(problem.kind, problem.dtype, problem.nx, problem.ref_precision)
        while want > 1 and problem.nz < want:
            want = 2 if want == 3 else want // 2
        temporal = 1
        if dev.type == "cuda" and want > 1 and native().hip_supports_steps(problem.kind, problem.dtype, problem.nx,
                                                                         problem.ny, problem.nz, want, want,
                                                                         problem.ref_precision):
            temporal = want
    lay = FieldLayout.make(problem, halo=max(1, temporal))
    a = alloc_field(lay, dev)
    b = alloc_field(lay, dev)
    dense_to_field(problem, g.to(TORCH_DTYPE[lay.dtype]), lay, a)
    left = steps
    while left > 0:
        k = temporal if left >= temporal else 1
        apply_stencil(problem, lay, a, b, steps=k)
        a, b = b, a
        left -= k
    out = field_to_dense(lay, a)
    return out.squeeze(1) if squeeze else out

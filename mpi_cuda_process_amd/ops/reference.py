"""Plain-PyTorch reference implementations of every stencil (the test oracle for the HIP kernels).

Each function takes a dense global grid ``u`` of shape ``(nz, ny, nx)`` (2D problems:
``(h, 1, w)``) and returns one updated grid. Global-boundary cells are held (Dirichlet /
dead frame), exactly the engine's semantics. These use ordinary tensor ops (no fused multiply-add),
so against the kernels they agree to rounding, not bitwise; the CPU oracle in the native core is
the bitwise reference.
"""

from __future__ import annotations

import torch


def heat7(u: torch.Tensor, r: float = 1.0 / 6.0) -> torch.Tensor:
    out = u.clone()
    if min(u.shape) < 3:
        return out
    c = u[1:-1, 1:-1, 1:-1]
    s = (((((u[1:-1, 1:-1, :-2] + u[1:-1, 1:-1, 2:]) + u[1:-1, :-2, 1:-1]) + u[1:-1, 2:, 1:-1])
          + u[:-2, 1:-1, 1:-1]) + u[2:, 1:-1, 1:-1])
    out[1:-1, 1:-1, 1:-1] = c + r * (s - 6.0 * c)
    return out


def jacobi5(u: torch.Tensor, r: float = 0.25) -> torch.Tensor:
    """2D 5-point; ``u`` is (h, 1, w) or (h, w)."""
    squeeze = u.dim() == 2
    g = u if squeeze else u[:, 0, :]
    out = g.clone()
    if min(g.shape) >= 3:
        c = g[1:-1, 1:-1]
        s = ((g[1:-1, :-2] + g[1:-1, 2:]) + g[:-2, 1:-1]) + g[2:, 1:-1]
        out[1:-1, 1:-1] = c + r * (s - 4.0 * c)
    return out if squeeze else out.unsqueeze(1)


def box27(u: torch.Tensor, c0: float = 0.25, c1: float = 1.0 / 20.0, c2: float = 1.0 / 40.0,
          c3: float = 3.0 / 160.0) -> torch.Tensor:
    out = u.clone()
    if min(u.shape) < 3:
        return out
    nz, ny, nx = u.shape
    faces = torch.zeros_like(u[1:-1, 1:-1, 1:-1])
    edges = torch.zeros_like(faces)
    corners = torch.zeros_like(faces)
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                k = abs(dz) + abs(dy) + abs(dx)
                if k == 0:
                    continue
                v = u[1 + dz:nz - 1 + dz, 1 + dy:ny - 1 + dy, 1 + dx:nx - 1 + dx]
                (faces if k == 1 else edges if k == 2 else corners).add_(v)
    out[1:-1, 1:-1, 1:-1] = c0 * u[1:-1, 1:-1, 1:-1] + c1 * faces + c2 * edges + c3 * corners
    return out


def life(u: torch.Tensor) -> torch.Tensor:
    """Game of Life B3/S23 with a held (dead) frame; ``u`` is (h, 1, w) or (h, w) uint8."""
    squeeze = u.dim() == 2
    g = (u if squeeze else u[:, 0, :]).to(torch.int32)
    out = g.clone()
    if min(g.shape) >= 3:
        h, w = g.shape
        n = torch.zeros_like(g[1:-1, 1:-1])
        for dz in (-1, 0, 1):
            for dx in (-1, 0, 1):
                if dz == 0 and dx == 0:
                    continue
                n += g[1 + dz:h - 1 + dz, 1 + dx:w - 1 + dx]
        alive = g[1:-1, 1:-1]
        out[1:-1, 1:-1] = ((n == 3) | ((n == 2) & (alive == 1))).to(torch.int32)
    out = out.to(torch.uint8)
    return out if squeeze else out.unsqueeze(1)


def step(kind: str, u: torch.Tensor, **coef) -> torch.Tensor:
    if kind == "heat7":
        r = coef.get("r", -1.0)
        return heat7(u, 1.0 / 6.0 if r is None or r < 0 else r)
    if kind == "jacobi5":
        r = coef.get("r", -1.0)
        return jacobi5(u, 0.25 if r is None or r < 0 else r)
    if kind == "box27":
        return box27(u, coef.get("c0", 0.25), coef.get("c1", 0.05), coef.get("c2", 0.025),
                     coef.get("c3", 3.0 / 160.0))
    if kind == "life":
        return life(u)
    raise ValueError(kind)


def run(kind: str, u: torch.Tensor, steps: int, **coef) -> torch.Tensor:
    for _ in range(steps):
        u = step(kind, u, **coef)
    return u


def residual(u_old: torch.Tensor, u_new: torch.Tensor) -> float:
    d = u_new.to(torch.float64) - u_old.to(torch.float64)
    return float(torch.sqrt((d * d).sum()))

"""Problem ("model") families of the stencil engine.

A :class:`Problem` names the stencil, the grid, the element type, the update coefficients and
the default initial condition. Families (reference parity in brackets):

* :func:`mdf2d`   — 2D 5-point heat / Jacobi, Dirichlet edges = 100, interior 0
  [MDF_kernel.cu:10-22 update, :88-99 initial grid]
* :func:`life2d`  — Conway's Game of Life, Moore-8, B3/S23, dead frame, density 0.15
  [kernel.cu:10-68 update, :131-146 initial grid]
* :func:`heat3d`  — 3D 7-point heat / Jacobi (headline benchmark, BASELINE.json configs 2, 3, 5)
* :func:`box27`   — 3D 27-point weighted stencil (BASELINE.json config 4)

2D grids are stored as ``nx = w, ny = 1, nz = h``: rows are the slab axis, exactly like the
reference's row split (MDF_kernel.cu:30,54).
"""

from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Optional

KINDS = ("jacobi5", "life", "heat7", "box27")


@dataclass(frozen=True)
class InitCondition:
    kind: str = "random"  # constant | dirichlet | random | life | compat (GoL glibc rand, host)
    seed: int = 1
    lo: float = 0.0
    hi: float = 1.0
    value: float = 0.0
    edge: float = 100.0
    interior: float = 0.0
    density: float = 0.15


@dataclass(frozen=True)
class Problem:
    kind: str
    nx: int
    ny: int
    nz: int
    dtype: str = "f32"
    r: float = -1.0  # 5/7-pt rate; < 0 -> 1/(2d) (Jacobi)
    c0: float = 0.25
    c1: float = 1.0 / 20.0
    c2: float = 1.0 / 40.0
    c3: float = 3.0 / 160.0
    # 2D MDF: evaluate the update exactly as the reference does (fp32 sum, fp64 scale and add;
    # MDF_kernel.cu:20) instead of wholly in the field type; single-step sweeps only
    ref_precision: bool = False
    init: InitCondition = field(default_factory=InitCondition)

    def __post_init__(self):
        if self.kind not in KINDS:
            raise ValueError("unknown stencil kind %r (one of %s)" % (self.kind, ", ".join(KINDS)))
        if self.kind in ("jacobi5", "life") and self.ny != 1:
            raise ValueError("2D problems use ny == 1 (nx = width, nz = height)")
        if self.kind == "life" and self.dtype != "u8":
            raise ValueError("life cells are u8")
        if self.kind != "life" and self.dtype not in ("f32", "f64"):
            raise ValueError("stencil dtype must be f32 or f64")
        for n in (self.nx, self.ny, self.nz):
            if n < 1:
                raise ValueError("grid extents must be positive")

    @property
    def dims(self) -> int:
        return 2 if self.kind in ("jacobi5", "life") else 3

    @property
    def cells(self) -> int:
        return self.nx * self.ny * self.nz

    @property
    def rate(self) -> float:
        if self.r >= 0:
            return self.r
        return 0.25 if self.kind == "jacobi5" else 1.0 / 6.0

    @property
    def bytes_per_cell_per_step(self) -> int:
        """Minimum HBM traffic of one sweep (one read + one write of every cell)."""
        return 2 * {"f32": 4, "f64": 8, "u8": 1}[self.dtype]

    def with_init(self, **kw) -> "Problem":
        return replace(self, init=replace(self.init, **kw))

    def coef_kwargs(self) -> dict:
        return dict(r=self.r, c0=self.c0, c1=self.c1, c2=self.c2, c3=self.c3, ref_precision=self.ref_precision)

    def describe(self) -> str:
        shape = "%dx%d" % (self.nz, self.nx) if self.dims == 2 else "%dx%dx%d" % (self.nx, self.ny, self.nz)
        return "%s %s %s" % (self.kind, shape, self.dtype)


def mdf2d(h: int = 256, w: int = 256, dtype: str = "f32", r: float = 0.25,
          init: Optional[InitCondition] = None, ref_precision: bool = False) -> Problem:
    """2D 5-point MDF (finite-difference) heat / Jacobi problem, Dirichlet edges 100.
    ``ref_precision`` pins the reference's mixed fp32/fp64 evaluation of the update."""
    return Problem("jacobi5", nx=w, ny=1, nz=h, dtype=dtype, r=r, ref_precision=ref_precision,
                   init=init or InitCondition(kind="dirichlet", edge=100.0, interior=0.0))


def life2d(h: int = 256, w: int = 256, density: float = 0.15, seed: int = 1,
           init: Optional[InitCondition] = None) -> Problem:
    """Conway's Game of Life on an h x w board with a dead frame."""
    return Problem("life", nx=w, ny=1, nz=h, dtype="u8",
                   init=init or InitCondition(kind="life", density=density, seed=seed))


def heat3d(n: int = 512, nx: Optional[int] = None, ny: Optional[int] = None, nz: Optional[int] = None,
           dtype: str = "f32", r: float = -1.0, init: Optional[InitCondition] = None) -> Problem:
    """3D 7-point heat / Jacobi problem on an nx x ny x nz grid (default n^3)."""
    return Problem("heat7", nx=nx or n, ny=ny or n, nz=nz or n, dtype=dtype, r=r,
                   init=init or InitCondition(kind="random", seed=1))


def box27(n: int = 512, nx: Optional[int] = None, ny: Optional[int] = None, nz: Optional[int] = None,
          dtype: str = "f32", c0: float = 0.25, c1: float = 1.0 / 20.0, c2: float = 1.0 / 40.0,
          c3: float = 3.0 / 160.0, init: Optional[InitCondition] = None) -> Problem:
    """3D 27-point weighted stencil u' = c0 u + c1 faces + c2 edges + c3 corners."""
    return Problem("box27", nx=nx or n, ny=ny or n, nz=nz or n, dtype=dtype, c0=c0, c1=c1, c2=c2,
                   c3=c3, init=init or InitCondition(kind="random", seed=1))


def from_name(kind: str, **kw) -> Problem:
    aliases = {"5": "jacobi5", "mdf": "jacobi5", "jacobi5": "jacobi5", "life": "life", "gol": "life",
               "7": "heat7", "heat7": "heat7", "jacobi7": "heat7", "27": "box27", "box27": "box27"}
    k = aliases.get(str(kind))
    if k is None:
        raise ValueError("unknown stencil %r" % kind)
    return {"jacobi5": mdf2d, "life": life2d, "heat7": heat3d, "box27": box27}[k](**kw)


__all__ = ["Problem", "InitCondition", "mdf2d", "life2d", "heat3d", "box27", "from_name", "KINDS"]

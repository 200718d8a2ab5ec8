"""HIP kernel numerics on the MI355X (tier T2 of SURVEY §4.3).

Every hand-written gfx950 kernel (tuned 2.5D z-march and naive one-cell-per-lane) is compared
(a) against the plain-PyTorch fp32/fp64 reference of the same op (tolerance) and (b) bitwise
against the native CPU oracle, which shares the point arithmetic. Odd sizes (non-multiples of the
tile) catch the floored-grid class of bug (reference D10).
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from mpi_cuda_process_amd import models  # noqa: E402
from mpi_cuda_process_amd.ops import (FieldLayout, alloc_field, apply_stencil, init_field,  # noqa: E402
                                      reference, set_kernel_variant)

CASES = [
    models.heat3d(nx=70, ny=33, nz=29),
    models.heat3d(nx=1100, ny=12, nz=9),  # 4 waves along x, ragged last tile
    models.heat3d(nx=300, ny=17, nz=11),  # 2 waves along x
    models.heat3d(nx=70, ny=33, nz=29, dtype="f64"),
    models.box27(nx=70, ny=21, nz=13),
    models.box27(nx=600, ny=9, nz=7),
    models.box27(nx=70, ny=21, nz=13, dtype="f64"),
    models.mdf2d(h=37, w=70),
    models.mdf2d(h=37, w=1500, dtype="f64"),
    models.life2d(h=41, w=77),
    models.life2d(h=23, w=2100),
]


def _ids(p):
    return p.describe().replace(" ", "_")


def _one_step(prob, device, variant="auto"):
    lay = FieldLayout.make(prob)
    src = alloc_field(lay, device)
    dst = alloc_field(lay, device)
    init_field(prob, lay, src)
    set_kernel_variant(variant if device != "cpu" else "auto")
    try:
        apply_stencil(prob, lay, src, dst)
    finally:
        set_kernel_variant("auto")
    if device != "cpu":
        torch.cuda.synchronize()
    return lay, src, dst


@pytest.mark.parametrize("prob", CASES, ids=_ids)
@pytest.mark.parametrize("variant", ["tuned", "naive"])
def test_kernel_matches_torch_reference(hip, prob, variant):
    lay, src, dst = _one_step(prob, "cuda", variant)
    u = src[lay.owned, :, : lay.nx]
    got = dst[lay.owned, :, : lay.nx]
    ref = reference.step(prob.kind, u.double() if prob.dtype != "u8" else u, **prob.coef_kwargs())
    if prob.dtype == "u8":
        assert torch.equal(got, ref)
    else:
        tol = 2e-6 if prob.dtype == "f32" else 1e-13
        err = (got.double() - ref).abs().max().item()
        assert err < tol, err


@pytest.mark.parametrize("prob", CASES, ids=_ids)
@pytest.mark.parametrize("variant", ["tuned", "naive"])
def test_kernel_bitwise_vs_cpu_oracle(hip, prob, variant):
    lay, _, dst_g = _one_step(prob, "cuda", variant)
    _, _, dst_c = _one_step(prob, "cpu")
    g = dst_g[lay.owned, :, : lay.nx].cpu()
    c = dst_c[lay.owned, :, : lay.nx]
    assert torch.equal(g, c), "max diff %g" % (g.double() - c.double()).abs().max().item()


@pytest.mark.parametrize("prob", [CASES[0], CASES[4], CASES[7], CASES[9]], ids=_ids)
def test_region_split_equals_full(hip, prob):
    """Interior + two boundary-plane launches == one full launch (the engine's split)."""
    lay, src, full = _one_step(prob, "cuda")
    parts = alloc_field(lay, "cuda")
    h, n = lay.halo, lay.z1 - lay.z0
    apply_stencil(prob, lay, src, parts, h, h + 1)
    apply_stencil(prob, lay, src, parts, h + n - 1, h + n)
    apply_stencil(prob, lay, src, parts, h + 1, h + n - 1)
    torch.cuda.synchronize()
    assert torch.equal(parts[lay.owned, :, : lay.nx], full[lay.owned, :, : lay.nx])


@pytest.mark.parametrize("prob", [CASES[0], CASES[3], CASES[4], CASES[7], CASES[9]], ids=_ids)
def test_residual_accumulator(hip, prob):
    lay = FieldLayout.make(prob)
    src = alloc_field(lay, "cuda")
    dst = alloc_field(lay, "cuda")
    init_field(prob, lay, src)
    acc = torch.zeros((), dtype=torch.float64, device="cuda")
    apply_stencil(prob, lay, src, dst, resid=acc)
    torch.cuda.synchronize()
    u0 = src[lay.owned, :, : lay.nx].double()
    u1 = dst[lay.owned, :, : lay.nx].double()
    want = float(((u1 - u0) ** 2).sum())
    assert abs(acc.item() - want) <= 1e-9 * max(1.0, want)


def test_init_matches_cpu(hip):
    for prob in (models.heat3d(nx=70, ny=9, nz=5), models.life2d(h=20, w=90), models.mdf2d(h=10, w=20)):
        lay = FieldLayout.make(prob, 2, 4)
        g = alloc_field(lay, "cuda")
        c = alloc_field(lay, "cpu")
        init_field(prob, lay, g)
        init_field(prob, lay, c)
        torch.cuda.synchronize()
        assert torch.equal(g.cpu()[:, :, : lay.nx], c[:, :, : lay.nx])


def test_heat7_large_plane_tuned(hip):
    """A 1024-wide plane (the headline's row width) through the tuned kernel, several chunks."""
    prob = models.heat3d(nx=1024, ny=64, nz=40)
    lay, src, dst = _one_step(prob, "cuda", "tuned")
    _, _, ref = _one_step(prob, "cuda", "naive")
    assert torch.equal(dst[lay.owned, :, : lay.nx], ref[lay.owned, :, : lay.nx])
    assert np.isfinite(dst.cpu().numpy()).all()

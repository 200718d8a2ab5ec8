"""Temporal blocking (2 fused Jacobi steps per sweep) on the MI355X: bitwise equal to two single
steps of the naive kernel and of the CPU oracle, for whole grids and for the engine's regions."""

import pytest
import torch

pytestmark = pytest.mark.gpu

from mpi_cuda_process_amd import models, native  # noqa: E402
from mpi_cuda_process_amd.ops import (FieldLayout, alloc_field, apply_stencil, init_field,  # noqa: E402
                                      set_kernel_variant)

CASES = [models.heat3d(nx=1024, ny=37, nz=23), models.heat3d(nx=700, ny=19, nz=15),
         models.heat3d(nx=256, ny=9, nz=12), models.heat3d(nx=500, ny=21, nz=11, dtype="f64"),
         models.heat3d(nx=64, ny=64, nz=9, r=0.1),
         # rows wider than one block: overlapping x tiles (3 tiles f32, 3 tiles f64, a 2-tile remainder)
         models.heat3d(nx=2048, ny=13, nz=11), models.heat3d(nx=1100, ny=9, nz=9, dtype="f64"),
         models.heat3d(nx=1030, ny=7, nz=8),
         # 2D 5-pt MDF (rows are planes): several segments, a ragged last one, fp64
         models.mdf2d(h=37, w=1000), models.mdf2d(h=21, w=300, dtype="f64"), models.mdf2d(h=9, w=64),
         # Game of Life (u8 SWAR): several 1024-cell segments, ragged edges
         models.life2d(h=40, w=3000), models.life2d(h=17, w=1024), models.life2d(h=9, w=100),
         # 27-point (partial sums through both levels): 4 / 2 / 1 waves across the row, fp64
         models.box27(nx=1024, ny=11, nz=9), models.box27(nx=512, ny=21, nz=15),
         models.box27(nx=300, ny=9, nz=12, dtype="f64"), models.box27(nx=64, ny=40, nz=10)]


def _two_single_steps(prob, lay, src, device):
    a = alloc_field(lay, device)
    b = alloc_field(lay, device)
    a.copy_(src)
    b.copy_(src)
    # single steps over owned planes only is not enough: the fused sweep also needs u1 on the
    # ghost planes, so compare over a full-grid layout where every plane is owned
    apply_stencil(prob, lay, a, b)
    c = alloc_field(lay, device)
    c.copy_(b)
    res = torch.zeros((), dtype=torch.float64, device=device)
    apply_stencil(prob, lay, b, c, resid=res)
    return c, res


@pytest.mark.parametrize("prob", CASES, ids=lambda p: p.describe().replace(" ", "_"))
@pytest.mark.parametrize("tbry", ["1", "2"])
def test_fused_two_steps_bitwise(hip, prob, tbry, knob):
    """The default two-step dispatch (heat7_tbk for rows within one block, heat7_tb2 x tiles for
    wider rows, jacobi5_tb2, life_tb2, box27_tb2) == two naive single steps and the CPU oracle;
    MDFX_TB_RY 1 / 2 rows per tile for the x-tiled and 27-point kernels."""
    knob("MDFX_TB_RY", tbry)
    lay = FieldLayout.make(prob, halo=2)
    src = alloc_field(lay, "cuda")
    init_field(prob, lay, src)
    fused = alloc_field(lay, "cuda")
    res = torch.zeros((), dtype=torch.float64, device="cuda")
    apply_stencil(prob, lay, src, fused, steps=2, resid=res)
    set_kernel_variant("naive")
    try:
        ref, ref_res = _two_single_steps(prob, lay, src, "cuda")
    finally:
        set_kernel_variant("auto")
    torch.cuda.synchronize()
    o = lay.owned
    assert torch.equal(fused[o, :, :lay.nx], ref[o, :, :lay.nx])
    # CPU oracle fused path agrees bitwise too
    cpu_src = src.cpu()
    cpu_out = alloc_field(lay, "cpu")
    apply_stencil(prob, lay, cpu_src, cpu_out, steps=2)
    assert torch.equal(fused[o, :, :lay.nx].cpu(), cpu_out[o, :, :lay.nx])
    # the fused residual is that of the second step (summation order differs)
    assert res.item() > 0 and abs(res.item() - ref_res.item()) <= 1e-9 * ref_res.item()


BOX27 = [models.box27(nx=1024, ny=11, nz=9), models.box27(nx=512, ny=21, nz=15),
         models.box27(nx=300, ny=9, nz=12, dtype="f64"), models.box27(nx=64, ny=40, nz=10),
         models.box27(nx=500, ny=30, nz=13, dtype="f64", c0=0.3, c1=0.05, c2=0.02, c3=0.01),
         models.box27(nx=200, ny=5, nz=9)]


@pytest.mark.parametrize("prob", BOX27, ids=lambda p: p.describe().replace(" ", "_"))
@pytest.mark.parametrize("tbry", ["0", "1"])
def test_box27_fused_kernels_bitwise(hip, prob, tbry, knob):
    """Both fused 27-point kernels (fp32: box27_tb2 in the natural layout with the 2-plane unroll,
    2 rows per tile or MDFX_TB_RY=1; fp64: box27_tbk with 4 rows per tile, 1 on short columns) ==
    two naive single steps, bitwise, with the residual of step 2."""
    knob("MDFX_TB_RY", tbry)
    lay = FieldLayout.make(prob, halo=2)
    src = alloc_field(lay, "cuda")
    init_field(prob, lay, src)
    fused = alloc_field(lay, "cuda")
    res = torch.zeros((), dtype=torch.float64, device="cuda")
    apply_stencil(prob, lay, src, fused, steps=2, resid=res)
    set_kernel_variant("naive")
    try:
        ref, ref_res = _two_single_steps(prob, lay, src, "cuda")
    finally:
        set_kernel_variant("auto")
    torch.cuda.synchronize()
    o = lay.owned
    assert torch.equal(fused[o, :, :lay.nx], ref[o, :, :lay.nx])
    assert res.item() > 0 and abs(res.item() - ref_res.item()) <= 1e-9 * ref_res.item()


def test_fused_region_on_a_slab_with_ghosts(hip):
    """A middle slab (z0 > 0, z1 < nz) with 2 ghost planes each side, interior + boundary regions."""
    prob = models.heat3d(nx=512, ny=16, nz=30)
    full = FieldLayout.make(prob, halo=2)
    g = alloc_field(full, "cuda")
    init_field(prob, full, g)
    ref = alloc_field(full, "cuda")
    apply_stencil(prob, full, g, ref, steps=2)
    lay = FieldLayout.make(prob, 10, 20, halo=2)
    src = alloc_field(lay, "cuda")
    init_field(prob, lay, src)  # ghosts from the global index == the neighbours' planes
    out = alloc_field(lay, "cuda")
    h = lay.halo
    apply_stencil(prob, lay, src, out, h, h + 2, steps=2)
    apply_stencil(prob, lay, src, out, h + 8, h + 10, steps=2)
    apply_stencil(prob, lay, src, out, h + 2, h + 8, steps=2)
    torch.cuda.synchronize()
    assert torch.equal(out[h:h + 10, :, :512], ref[10 + 2:20 + 2, :, :512])


import numpy as np  # noqa: E402

import mpi_cuda_process_amd as mm  # noqa: E402


def _sim(prob, steps, **kw):
    with mm.Simulation(prob, device="hip", **kw) as sim:
        sim.init()
        sim.run(steps)
        sim.synchronize()
        return sim.gather(), sim.residual


@pytest.mark.parametrize("ranks", [1, 2, 4])
def test_engine_temporal2_equals_single_steps(hip, ranks):
    prob = mm.heat3d(nx=1024, ny=24, nz=40)
    ref, _ = _sim(prob, 9, ranks=1)
    got, _ = _sim(prob, 9, ranks=ranks, temporal=2)
    assert np.array_equal(ref, got)


def test_engine_temporal2_graph_and_residual(hip):
    prob = mm.heat3d(nx=512, ny=32, nz=33, dtype="f64")
    ref, rr = _sim(prob, 12, ranks=1, residual_every=6)
    got, rg = _sim(prob, 12, ranks=1, temporal=2, graph=True, residual_every=6)
    assert np.array_equal(ref, got) and abs(rr - rg) <= 1e-9 * rr
    got2, _ = _sim(prob, 12, ranks=3, temporal=2, overlap=False, sync_debug=True)
    assert np.array_equal(ref, got2)


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_engine_temporal2_wide_rows(hip, dtype):
    """2048-wide rows (the 2048^3 fp64 config's width) run x-tiled and stay bitwise."""
    prob = mm.heat3d(nx=2048, ny=12, nz=20, dtype=dtype)
    ref, _ = _sim(prob, 7, ranks=1)
    got, _ = _sim(prob, 7, ranks=2, temporal=2)
    assert np.array_equal(ref, got)


@pytest.mark.parametrize("ranks", [1, 3])
def test_engine_temporal2_mdf2d(hip, ranks):
    """The reference's own 2D MDF problem, fused: equal to single steps for any slab count."""
    prob = mm.mdf2d(h=300, w=777)
    ref, rr = _sim(prob, 11, ranks=1, residual_every=11)
    got, rg = _sim(prob, 11, ranks=ranks, temporal=2, residual_every=11)
    assert np.array_equal(ref, got) and abs(rr - rg) <= 1e-9 * rr


@pytest.mark.parametrize("ranks", [1, 4])
def test_engine_temporal2_life(hip, ranks):
    prob = mm.life2d(h=333, w=2100)
    ref, rr = _sim(prob, 13, ranks=1, residual_every=13)
    got, rg = _sim(prob, 13, ranks=ranks, temporal=2, residual_every=13)
    assert np.array_equal(ref, got) and rr == rg


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_engine_temporal2_box27(hip, dtype):
    prob = mm.box27(nx=512, ny=40, nz=50, dtype=dtype)
    ref, rr = _sim(prob, 9, ranks=1, residual_every=9)
    got, rg = _sim(prob, 9, ranks=3, temporal=2, residual_every=9)
    assert np.array_equal(ref, got) and abs(rr - rg) <= 1e-9 * rr


DEEP = [models.mdf2d(h=45, w=1000), models.mdf2d(h=33, w=300, dtype="f64"), models.life2d(h=50, w=3000),
        models.life2d(h=19, w=100),
        # the reference's mixed fp32 / fp64 evaluation (MDF_kernel.cu:20): at its r = 0.25 through the
        # plain kernels (StencilSpec::mixed_update), at other r through jacobi5_tbk REF
        models.mdf2d(h=45, w=1000, ref_precision=True).with_init(kind="random", seed=5, lo=-50.0, hi=150.0),
        models.mdf2d(h=23, w=130, ref_precision=True),
        models.mdf2d(h=45, w=1000, r=0.2, ref_precision=True).with_init(kind="random", seed=5, lo=-50.0, hi=150.0),
        models.mdf2d(h=23, w=130, r=0.15, ref_precision=True)]


@pytest.mark.parametrize("prob", DEEP, ids=lambda p: p.describe().replace(" ", "_"))
@pytest.mark.parametrize("k", [2, 3, 4, 6, 8])
def test_deep_fused_steps_bitwise(hip, prob, k):
    """K fused steps per sweep (K = 2: jacobi5_tb2 / life_tb2, or jacobi5_tbk REF where the mixed
    update can change a bit; deeper: the overlapping-segment kernels jacobi5_tbk / life_bits) == K
    naive single steps, bitwise."""
    for force in (0,):
        lay = FieldLayout.make(prob, halo=k)
        src = alloc_field(lay, "cuda")
        init_field(prob, lay, src)
        fused = alloc_field(lay, "cuda")
        res = torch.zeros((), dtype=torch.float64, device="cuda")
        apply_stencil(prob, lay, src, fused, steps=k, resid=res)
        set_kernel_variant("naive")
        try:
            cur = alloc_field(lay, "cuda")
            cur.copy_(src)
            ref_res = torch.zeros((), dtype=torch.float64, device="cuda")
            for i in range(k):
                nxt = alloc_field(lay, "cuda")
                nxt.copy_(cur)
                apply_stencil(prob, lay, cur, nxt, resid=ref_res if i == k - 1 else None)
                cur = nxt
        finally:
            set_kernel_variant("auto")
        torch.cuda.synchronize()
        o = lay.owned
        assert torch.equal(fused[o, :, :lay.nx], cur[o, :, :lay.nx]), (k, force)
        assert abs(res.item() - ref_res.item()) <= 1e-9 * max(1.0, ref_res.item())


def test_ref_precision_at_power_of_two_rate_is_the_field_type_update(hip):
    """At the reference's r = 0.25 its mixed fp32 / fp64 update rounds exactly like the fp32 fma
    update (proof: StencilSpec::mixed_update), so ref_precision runs the plain fused kernels; the
    naive kernel evaluates the reference's expression literally and must agree bit for bit."""
    out = {}
    for ref in (False, True):
        prob = models.mdf2d(h=64, w=1000, ref_precision=ref).with_init(kind="random", seed=3, lo=-50.0, hi=150.0)
        lay = FieldLayout.make(prob, halo=8)
        src = alloc_field(lay, "cuda")
        init_field(prob, lay, src)
        dst = alloc_field(lay, "cuda")
        apply_stencil(prob, lay, src, dst, steps=8)
        out[ref] = dst[lay.owned, :, :lay.nx].clone()
        if ref:
            set_kernel_variant("naive")
            try:
                cur = src.clone()
                for _ in range(8):
                    nxt = cur.clone()
                    apply_stencil(prob, lay, cur, nxt)
                    cur = nxt
            finally:
                set_kernel_variant("auto")
            out["naive"] = cur[lay.owned, :, :lay.nx].clone()
    assert torch.equal(out[False], out[True]) and torch.equal(out[True], out["naive"])


LIFE_DEEP = [models.life2d(h=50, w=3000), models.life2d(h=19, w=100), models.life2d(h=40, w=2049),
             models.life2d(h=70, w=64, density=0.4)]


@pytest.mark.parametrize("prob", LIFE_DEEP, ids=lambda p: p.describe().replace(" ", "_"))
@pytest.mark.parametrize("k", [2, 3, 4, 6, 8, 12, 16])
def test_life_kernels_bitwise(hip, prob, k):
    """K Life generations per sweep (two: life_tb2; deeper: the bit-sliced life_bits, up to 16) == K
    naive generations, bitwise, with the change count of the last."""
    for bits in (1,):
        lay = FieldLayout.make(prob, halo=k)
        src = alloc_field(lay, "cuda")
        init_field(prob, lay, src)
        fused = alloc_field(lay, "cuda")
        res = torch.zeros((), dtype=torch.float64, device="cuda")
        apply_stencil(prob, lay, src, fused, steps=k, resid=res)
        set_kernel_variant("naive")
        try:
            cur = alloc_field(lay, "cuda")
            cur.copy_(src)
            ref_res = torch.zeros((), dtype=torch.float64, device="cuda")
            for i in range(k):
                nxt = alloc_field(lay, "cuda")
                nxt.copy_(cur)
                apply_stencil(prob, lay, cur, nxt, resid=ref_res if i == k - 1 else None)
                cur = nxt
        finally:
            set_kernel_variant("auto")
        torch.cuda.synchronize()
        o = lay.owned
        assert torch.equal(fused[o, :, :lay.nx], cur[o, :, :lay.nx]), (k, bits)
        assert res.item() == ref_res.item(), (k, bits)


@pytest.mark.parametrize("prob,k", [(mm.mdf2d(h=400, w=1500), 8), (mm.mdf2d(h=200, w=700, dtype="f64"), 4),
                                    (mm.life2d(h=300, w=5000), 4), (mm.life2d(h=300, w=2000), 6),
                                    (mm.life2d(h=300, w=4100), 16), (mm.life2d(h=200, w=1000), 12)])
def test_engine_deep_temporal_2d(hip, prob, k):
    ref, rr = _sim(prob, 37, ranks=1, residual_every=9)
    got, rg = _sim(prob, 37, ranks=4, temporal=k, residual_every=9)
    assert np.array_equal(ref, got) and abs(rr - rg) <= 1e-9 * max(1.0, rr)


# 3D 7-point deep temporal blocking (heat7_tbk, streaming per-level partial sums): rows that fit
# one block (1024 fp32 / 512 fp64) with 4 / 2 / 1 waves across the row, ragged widths, y / z edges
DEEP3D = [models.heat3d(nx=1024, ny=37, nz=23), models.heat3d(nx=700, ny=19, nz=15),
          models.heat3d(nx=256, ny=9, nz=12), models.heat3d(nx=500, ny=21, nz=11, dtype="f64"),
          models.heat3d(nx=64, ny=64, nz=9, r=0.1), models.heat3d(nx=1000, ny=5, nz=14),
          models.heat3d(nx=300, ny=40, nz=10, dtype="f64")]


@pytest.mark.parametrize("prob", DEEP3D, ids=lambda p: p.describe().replace(" ", "_"))
@pytest.mark.parametrize("k", [2, 3, 4])
def test_heat7_deep_fused_bitwise(hip, prob, k):
    """The 3D 7-point's K fused steps per sweep (K = 2: heat7_tbk, 4 rows per tile, 1 on short
    columns; K = 3 / 4: heat7_wxk / heat7_wtk) == K naive single steps, bitwise, with the residual
    of step K."""
    ry = "auto"
    lay = FieldLayout.make(prob, halo=k)
    src = alloc_field(lay, "cuda")
    init_field(prob, lay, src)
    fused = alloc_field(lay, "cuda")
    res = torch.zeros((), dtype=torch.float64, device="cuda")
    apply_stencil(prob, lay, src, fused, steps=k, resid=res)
    set_kernel_variant("naive")
    try:
        cur = alloc_field(lay, "cuda")
        cur.copy_(src)
        ref_res = torch.zeros((), dtype=torch.float64, device="cuda")
        for i in range(k):
            nxt = alloc_field(lay, "cuda")
            nxt.copy_(cur)
            apply_stencil(prob, lay, cur, nxt, resid=ref_res if i == k - 1 else None)
            cur = nxt
    finally:
        set_kernel_variant("auto")
    torch.cuda.synchronize()
    o = lay.owned
    assert torch.equal(fused[o, :, :lay.nx], cur[o, :, :lay.nx]), (k, ry)
    assert res.item() > 0 and abs(res.item() - ref_res.item()) <= 1e-9 * ref_res.item()


WIDE3D = [models.heat3d(nx=2048, ny=13, nz=11), models.heat3d(nx=1100, ny=9, nz=9, dtype="f64"),
          models.heat3d(nx=1030, ny=7, nz=8), models.heat3d(nx=2048, ny=21, nz=12, dtype="f64"),
          models.heat3d(nx=1300, ny=17, nz=10, r=0.1)]


@pytest.mark.parametrize("prob", WIDE3D, ids=lambda p: p.describe().replace(" ", "_"))
@pytest.mark.parametrize("tbry", ["1", "2"])
def test_heat7_xtiled_fused_bitwise(hip, prob, tbry, knob):
    """Rows wider than one block: heat7_tb2's x tiles (the edge waves recompute the neighbour
    tile's u1 column) == two naive single steps, bitwise, with the residual of step 2."""
    knob("MDFX_TB_RY", tbry)
    lay = FieldLayout.make(prob, halo=2)
    src = alloc_field(lay, "cuda")
    init_field(prob, lay, src)
    fused = alloc_field(lay, "cuda")
    res = torch.zeros((), dtype=torch.float64, device="cuda")
    apply_stencil(prob, lay, src, fused, steps=2, resid=res)
    set_kernel_variant("naive")
    try:
        ref, ref_res = _two_single_steps(prob, lay, src, "cuda")
    finally:
        set_kernel_variant("auto")
    torch.cuda.synchronize()
    o = lay.owned
    assert torch.equal(fused[o, :, :lay.nx], ref[o, :, :lay.nx]), tbry
    assert res.item() > 0 and abs(res.item() - ref_res.item()) <= 1e-9 * ref_res.item()


def test_heat7_deep_fused_regions_on_a_slab(hip):
    """A middle slab with 4 ghost planes: boundary + interior region launches == the whole grid."""
    prob = models.heat3d(nx=1024, ny=20, nz=40)
    full = FieldLayout.make(prob, halo=4)
    g = alloc_field(full, "cuda")
    init_field(prob, full, g)
    ref = alloc_field(full, "cuda")
    apply_stencil(prob, full, g, ref, steps=4)
    lay = FieldLayout.make(prob, 12, 30, halo=4)
    src = alloc_field(lay, "cuda")
    init_field(prob, lay, src)
    out = alloc_field(lay, "cuda")
    h = lay.halo
    apply_stencil(prob, lay, src, out, h, h + 4, steps=4)
    apply_stencil(prob, lay, src, out, h + 14, h + 18, steps=4)
    apply_stencil(prob, lay, src, out, h + 4, h + 14, steps=4)
    torch.cuda.synchronize()
    assert torch.equal(out[h:h + 18, :, :1024], ref[12 + 4:30 + 4, :, :1024])


@pytest.mark.parametrize("k,ranks", [(3, 1), (3, 3), (4, 1), (4, 4)])
def test_engine_deep_temporal_3d(hip, k, ranks):
    prob = mm.heat3d(nx=1024, ny=24, nz=60)
    ref, rr = _sim(prob, 23, ranks=1, residual_every=10)
    got, rg = _sim(prob, 23, ranks=ranks, temporal=k, residual_every=10)
    assert np.array_equal(ref, got) and abs(rr - rg) <= 1e-9 * rr


STALE_LDS = [models.heat3d(nx=256, ny=9, nz=12), models.heat3d(nx=500, ny=21, nz=11, dtype="f64"),
             models.heat3d(nx=700, ny=19, nz=15), models.heat3d(nx=1024, ny=12, nz=9),
             models.heat3d(nx=2048, ny=13, nz=11), models.box27(nx=300, ny=9, nz=12, dtype="f64"),
             models.box27(nx=1024, ny=11, nz=9), models.mdf2d(h=37, w=1000), models.life2d(h=40, w=3000)]


@pytest.mark.parametrize("prob", STALE_LDS, ids=lambda p: p.describe().replace(" ", "_"))
@pytest.mark.parametrize("k", [1, 2])
def test_kernels_never_read_stale_lds(hip, prob, k):
    """Every CU's LDS is filled with NaN right before the tuned kernel runs: a kernel that read LDS
    it had not written (e.g. a missing wave-seam at the global x boundary, held with a zero
    coefficient that cannot cancel NaN) would now differ from the naive single steps."""
    from mpi_cuda_process_amd import native

    lay = FieldLayout.make(prob, halo=k)
    src = alloc_field(lay, "cuda")
    init_field(prob, lay, src)
    out = alloc_field(lay, "cuda")
    torch.cuda.synchronize()
    native().poison_lds()
    apply_stencil(prob, lay, src, out, steps=k)
    set_kernel_variant("naive")
    try:
        cur = alloc_field(lay, "cuda")
        cur.copy_(src)
        for _ in range(k):
            nxt = alloc_field(lay, "cuda")
            nxt.copy_(cur)
            apply_stencil(prob, lay, cur, nxt)
            cur = nxt
    finally:
        set_kernel_variant("auto")
    torch.cuda.synchronize()
    o = lay.owned
    assert torch.equal(out[o, :, :lay.nx], cur[o, :, :lay.nx])


# heat7_wtk (wave-independent tiles: overlapping wave segments in x, recomputed y halo, streaming
# z levels, per-wave LDS-DMA slots): any row width, including rows wider than one block
WTK3D = DEEP3D + [models.heat3d(nx=2048, ny=13, nz=11), models.heat3d(nx=1100, ny=9, nz=9, dtype="f64"),
                  models.heat3d(nx=1030, ny=7, nz=8), models.heat3d(nx=8, ny=6, nz=9)]


@pytest.mark.parametrize("prob", [p for p in WTK3D if p.dtype == "f64"] + [models.heat3d(nx=300, ny=33, nz=9, dtype="f64")],
                         ids=lambda p: p.describe().replace(" ", "_"))
@pytest.mark.parametrize("k,wb", [(3, "4"), (3, "8"), (4, "4")])
@pytest.mark.parametrize("resid", [False, True])
def test_heat7_wtk_bitwise(hip, prob, k, wb, resid, knob):
    """heat7_wtk's K fused steps (fp64 only since round 6: the 3D 7-point kernel for K = 3 where
    heat7_wxk does not run, fp64 rows below 2048 cells, and any fp64 K = 3 / 4 under MDFX_H7_WXK=0)
    == K naive single steps, bitwise, with or without the
    residual of step K, in bands of 4 or 8 waves."""
    knob("MDFX_H7_WXK", 0)
    knob("MDFX_WTK_WB", wb)
    lay = FieldLayout.make(prob, halo=k)
    src = alloc_field(lay, "cuda")
    init_field(prob, lay, src)
    fused = alloc_field(lay, "cuda")
    res = torch.zeros((), dtype=torch.float64, device="cuda")
    apply_stencil(prob, lay, src, fused, steps=k, resid=res if resid else None)
    set_kernel_variant("naive")
    try:
        cur = alloc_field(lay, "cuda")
        cur.copy_(src)
        ref_res = torch.zeros((), dtype=torch.float64, device="cuda")
        for i in range(k):
            nxt = alloc_field(lay, "cuda")
            nxt.copy_(cur)
            apply_stencil(prob, lay, cur, nxt, resid=ref_res if i == k - 1 else None)
            cur = nxt
    finally:
        set_kernel_variant("auto")
    torch.cuda.synchronize()
    o = lay.owned
    assert torch.equal(fused[o, :, :lay.nx], cur[o, :, :lay.nx]), (k, wb)
    if resid:
        assert res.item() > 0 and abs(res.item() - ref_res.item()) <= 1e-9 * ref_res.item()


@pytest.mark.parametrize("prob", WTK3D + [models.heat3d(nx=700, ny=70, nz=12), models.heat3d(nx=300, ny=33, nz=9, dtype="f64")],
                         ids=lambda p: p.describe().replace(" ", "_"))
@pytest.mark.parametrize("k", [3, 4, 5])
@pytest.mark.parametrize("resid", [False, True])
def test_heat7_wxk_bitwise(hip, prob, k, resid, knob):
    """heat7_wxk (y halo exchanged between the waves of a band through the LDS seam table, one
    barrier per plane) == K naive single steps, bitwise, with the residual of step K, for every
    shipped band and row count, including bands taller than the grid and waves wholly outside it
    (K = 5: fp32 in rows of 2 cells per lane, fp64 in rows of 1 cell per lane)."""
    knob("MDFX_H7_WXK", 1)
    lay = FieldLayout.make(prob, halo=k)
    src = alloc_field(lay, "cuda")
    init_field(prob, lay, src)
    fused = alloc_field(lay, "cuda")
    res = torch.zeros((), dtype=torch.float64, device="cuda")
    apply_stencil(prob, lay, src, fused, steps=k, resid=res if resid else None)
    set_kernel_variant("naive")
    try:
        cur = src.clone()
        ref_res = torch.zeros((), dtype=torch.float64, device="cuda")
        for i in range(k):
            nxt = cur.clone()
            apply_stencil(prob, lay, cur, nxt, resid=ref_res if i == k - 1 else None)
            cur = nxt
    finally:
        set_kernel_variant("auto")
    torch.cuda.synchronize()
    o = lay.owned
    assert torch.equal(fused[o, :, :lay.nx], cur[o, :, :lay.nx]), k
    if resid:
        assert res.item() > 0 and abs(res.item() - ref_res.item()) <= 1e-9 * ref_res.item()


@pytest.mark.parametrize("resid", [False, True])
@pytest.mark.parametrize("nx,k", [(1024, 4), (2048, 5)])
def test_heat7_fp64_wide_rows_default_path(hip, resid, nx, k):
    """fp64 rows of 1024 cells take heat7_wxk at K = 4 by default (2 + 1-row bands), rows of 2048
    cells and more at K = 5 (1 cell per lane): the engine's default fused depth and kernel == K naive
    single steps, bitwise."""
    prob = models.heat3d(nx=nx, ny=23, nz=13, dtype="f64")
    assert native().hip_fused_depth(prob.kind, prob.dtype, prob.nx, False) == k
    lay = FieldLayout.make(prob, halo=k)
    src = alloc_field(lay, "cuda")
    init_field(prob, lay, src)
    fused = alloc_field(lay, "cuda")
    res = torch.zeros((), dtype=torch.float64, device="cuda")
    apply_stencil(prob, lay, src, fused, steps=k, resid=res if resid else None)
    set_kernel_variant("naive")
    try:
        cur = src.clone()
        ref_res = torch.zeros((), dtype=torch.float64, device="cuda")
        for i in range(k):
            nxt = cur.clone()
            apply_stencil(prob, lay, cur, nxt, resid=ref_res if i == k - 1 else None)
            cur = nxt
    finally:
        set_kernel_variant("auto")
    torch.cuda.synchronize()
    o = lay.owned
    assert torch.equal(fused[o, :, :lay.nx], cur[o, :, :lay.nx])
    if resid:
        assert res.item() > 0 and abs(res.item() - ref_res.item()) <= 1e-9 * ref_res.item()


B27X = [models.box27(n=40), models.box27(n=24, dtype="f64"), models.box27(nx=700, ny=37, nz=15),
        models.box27(nx=1030, ny=9, nz=12), models.box27(nx=300, ny=70, nz=10, dtype="f64"),
        models.box27(nx=8, ny=5, nz=9),
        # rows of 257..512 cells (3 overlapping x segments; round 3's x-pair kernel was removed)
        models.box27(nx=512, ny=29, nz=14), models.box27(nx=300, ny=17, nz=11), models.box27(nx=257, ny=9, nz=8),
        models.box27(nx=512, ny=5, nz=9), models.box27(nx=448, ny=40, nz=23),
        models.box27(nx=512, ny=13, nz=9, dtype="f64"), models.box27(nx=130, ny=21, nz=7, dtype="f64")]


@pytest.mark.parametrize("prob", B27X, ids=lambda p: p.describe().replace(" ", "_"))
@pytest.mark.parametrize("resid", [False, True])
def test_box27_wxk_bitwise(hip, prob, resid):
    """box27_wxk (27-point, K = 3, y halo exchanged through the LDS seam table, levels above the
    first one plane later) == 3 naive box27 steps, bitwise, with the residual of step 3."""
    k = 3
    lay = FieldLayout.make(prob, halo=k)
    src = alloc_field(lay, "cuda")
    init_field(prob, lay, src)
    fused = alloc_field(lay, "cuda")
    res = torch.zeros((), dtype=torch.float64, device="cuda")
    apply_stencil(prob, lay, src, fused, steps=k, resid=res if resid else None)
    set_kernel_variant("naive")
    try:
        cur = src.clone()
        ref_res = torch.zeros((), dtype=torch.float64, device="cuda")
        for i in range(k):
            nxt = cur.clone()
            apply_stencil(prob, lay, cur, nxt, resid=ref_res if i == k - 1 else None)
            cur = nxt
    finally:
        set_kernel_variant("auto")
    torch.cuda.synchronize()
    o = lay.owned
    assert torch.equal(fused[o, :, :lay.nx], cur[o, :, :lay.nx])
    if resid:
        assert res.item() > 0 and abs(res.item() - ref_res.item()) <= 1e-9 * ref_res.item()


@pytest.mark.parametrize("nx", [600, 480])
def test_box27_wxk_regions_and_engine(hip, knob, nx):
    """box27_wxk on a middle slab (both boundary regions in one launch + the interior) == the
    whole grid, and a 3-slab engine run at the 27-point's fused depth 3 == single steps."""
    k = 3
    prob = models.box27(nx=nx, ny=30, nz=40)
    full = FieldLayout.make(prob, halo=k)
    g = alloc_field(full, "cuda")
    init_field(prob, full, g)
    ref = alloc_field(full, "cuda")
    apply_stencil(prob, full, g, ref, steps=k)
    lay = FieldLayout.make(prob, 12, 30, halo=k)
    src = alloc_field(lay, "cuda")
    init_field(prob, lay, src)
    out = alloc_field(lay, "cuda")
    h = lay.halo
    res = torch.zeros((), dtype=torch.float64, device="cuda")
    apply_stencil(prob, lay, src, out, h, h + k, steps=k, second=(h + 18 - k, h + 18), resid=res)
    apply_stencil(prob, lay, src, out, h + k, h + 18 - k, steps=k, resid=res)
    torch.cuda.synchronize()
    assert torch.equal(out[h:h + 18, :, :nx], ref[12 + k:30 + k, :, :nx])
    # the two-region launch's residual == three single-region launches'
    res3 = torch.zeros((), dtype=torch.float64, device="cuda")
    out3 = alloc_field(lay, "cuda")
    for lo, hi in ((h, h + k), (h + 18 - k, h + 18), (h + k, h + 18 - k)):
        apply_stencil(prob, lay, src, out3, lo, hi, steps=k, resid=res3)
    torch.cuda.synchronize()
    assert res.item() > 0 and abs(res.item() - res3.item()) <= 1e-9 * res3.item()
    knob("MDFX_B27_WXK", 1)
    p3 = models.box27(nx=500, ny=33, nz=45)
    a, _ = _sim(p3, 6, ranks=1)
    b, _ = _sim(p3, 6, ranks=3, temporal=3)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("k,dtype", [(3, "f32"), (4, "f32"), (5, "f32"), (5, "f64")])
def test_heat7_wxk_regions_and_engine(hip, k, dtype, knob):
    """heat7_wxk on a middle slab: both boundary regions in one launch + the interior == the whole
    grid; and an engine run over 3 slabs with the wxk sweeps == single steps."""
    knob("MDFX_H7_WXK", 1)
    prob = models.heat3d(nx=1024, ny=20, nz=40, dtype=dtype)
    full = FieldLayout.make(prob, halo=k)
    g = alloc_field(full, "cuda")
    init_field(prob, full, g)
    ref = alloc_field(full, "cuda")
    apply_stencil(prob, full, g, ref, steps=k)
    lay = FieldLayout.make(prob, 12, 30, halo=k)
    src = alloc_field(lay, "cuda")
    init_field(prob, lay, src)
    out = alloc_field(lay, "cuda")
    h = lay.halo
    res = torch.zeros((), dtype=torch.float64, device="cuda")
    apply_stencil(prob, lay, src, out, h, h + k, steps=k, second=(h + 18 - k, h + 18), resid=res)
    apply_stencil(prob, lay, src, out, h + k, h + 18 - k, steps=k, resid=res)
    torch.cuda.synchronize()
    assert torch.equal(out[h:h + 18, :, :1024], ref[12 + k:30 + k, :, :1024])
    # the fused two-region launch's residual == three single-region launches' (a wrong residual from
    # the second region's tasks would show here)
    res3 = torch.zeros((), dtype=torch.float64, device="cuda")
    out3 = alloc_field(lay, "cuda")
    for lo, hi in ((h, h + k), (h + 18 - k, h + 18), (h + k, h + 18 - k)):
        apply_stencil(prob, lay, src, out3, lo, hi, steps=k, resid=res3)
    torch.cuda.synchronize()
    assert res.item() > 0 and abs(res.item() - res3.item()) <= 1e-9 * res3.item()
    p3 = models.heat3d(nx=600, ny=37, nz=45, dtype=dtype)
    a, _ = _sim(p3, 2 * k, ranks=1)
    b, _ = _sim(p3, 2 * k, ranks=3, temporal=k)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("k", [3, 4])
def test_heat7_wtk_regions_on_a_slab(hip, k):
    """heat7_wtk on a middle slab with K ghost planes: boundary + interior regions == whole grid."""
    prob = models.heat3d(nx=1024, ny=20, nz=40)
    full = FieldLayout.make(prob, halo=k)
    g = alloc_field(full, "cuda")
    init_field(prob, full, g)
    ref = alloc_field(full, "cuda")
    apply_stencil(prob, full, g, ref, steps=k)
    lay = FieldLayout.make(prob, 12, 30, halo=k)
    src = alloc_field(lay, "cuda")
    init_field(prob, lay, src)
    out = alloc_field(lay, "cuda")
    h = lay.halo
    apply_stencil(prob, lay, src, out, h, h + k, steps=k)
    apply_stencil(prob, lay, src, out, h + 18 - k, h + 18, steps=k)
    apply_stencil(prob, lay, src, out, h + k, h + 18 - k, steps=k)
    torch.cuda.synchronize()
    assert torch.equal(out[h:h + 18, :, :1024], ref[12 + k:30 + k, :, :1024])
    # both boundary regions in ONE call (one heat7_wtk launch), with their residual
    out2 = alloc_field(lay, "cuda")
    res2 = torch.zeros((), dtype=torch.float64, device="cuda")
    apply_stencil(prob, lay, src, out2, h, h + k, steps=k, second=(h + 18 - k, h + 18), resid=res2)
    res1 = torch.zeros((), dtype=torch.float64, device="cuda")
    out3 = alloc_field(lay, "cuda")
    apply_stencil(prob, lay, src, out3, h, h + k, steps=k, resid=res1)
    apply_stencil(prob, lay, src, out3, h + 18 - k, h + 18, steps=k, resid=res1)
    torch.cuda.synchronize()
    for lo, hi in ((h, h + k), (h + 18 - k, h + 18)):
        assert torch.equal(out2[lo:hi, :, :1024], out[lo:hi, :, :1024])
    assert res2.item() > 0 and abs(res2.item() - res1.item()) <= 1e-9 * res1.item()


@pytest.mark.parametrize("k,ranks,wxk,dtype", [(3, 1, "-1", "f32"), (3, 3, "-1", "f32"), (4, 2, "-1", "f32"),
                                              (3, 3, "-1", "f64"), (3, 3, "0", "f64"), (4, 2, "0", "f64")])
def test_engine_wtk_temporal_3d(hip, k, ranks, wxk, dtype, knob):
    """The engine's K-step sweeps (heat7_wxk by default; fp64 K = 3 at 1024-cell rows, and fp64 K =
    3 / 4 with MDFX_H7_WXK=0, through heat7_wtk) over 1-3 slabs with a residual every 10 steps ==
    single steps."""
    knob("MDFX_H7_WXK", wxk)
    prob = mm.heat3d(nx=1024, ny=24, nz=60, dtype=dtype)
    ref, rr = _sim(prob, 23, ranks=1, temporal=1, residual_every=10)
    got, rg = _sim(prob, 23, ranks=ranks, temporal=k, residual_every=10)
    assert np.array_equal(ref, got) and abs(rr - rg) <= 1e-9 * rr


@pytest.mark.parametrize("prob", [models.heat3d(nx=1024, ny=12, nz=11, dtype="f64"), models.heat3d(nx=500, ny=21, nz=11, dtype="f64")],
                         ids=lambda p: p.describe().replace(" ", "_"))
def test_wtk_never_reads_stale_lds(hip, prob):
    """heat7_wtk reads only LDS its own DMA filled: NaN-poisoned LDS does not change the result."""
    from mpi_cuda_process_amd import native

    k = 3
    lay = FieldLayout.make(prob, halo=k)
    src = alloc_field(lay, "cuda")
    init_field(prob, lay, src)
    out = alloc_field(lay, "cuda")
    torch.cuda.synchronize()
    native().poison_lds()
    apply_stencil(prob, lay, src, out, steps=k)
    set_kernel_variant("naive")
    try:
        cur = alloc_field(lay, "cuda")
        cur.copy_(src)
        for _ in range(k):
            nxt = alloc_field(lay, "cuda")
            nxt.copy_(cur)
            apply_stencil(prob, lay, cur, nxt)
            cur = nxt
    finally:
        set_kernel_variant("auto")
    torch.cuda.synchronize()
    o = lay.owned
    assert torch.equal(out[o, :, :lay.nx], cur[o, :, :lay.nx])

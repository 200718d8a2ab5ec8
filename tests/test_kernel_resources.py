"""Static resource check of every gfx950 kernel in libmdfx.so (VGPR / LDS / occupancy
checked in CI). Reads the AMDHSA metadata of the code objects; no GPU needed."""

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

from kernel_resources import kernel_isa, kernel_resources  # noqa: E402

LIB = os.path.join(ROOT, "mpi_cuda_process_amd", "lib", "libmdfx.so")


@pytest.fixture(scope="module")
def recs():
    if not os.path.exists(LIB):
        pytest.fail("libmdfx.so is not built (make -j8 all)")
    r = kernel_resources(LIB)
    assert len(r) > 50
    return {x["name"].split("(")[0].replace("void ", ""): x for x in r}


def test_no_kernel_spills_to_scratch(recs):
    # VGPR spills go to scratch memory (HBM round trips inside the z-march). SGPR spills land in
    # VGPR lanes (v_writelane / v_readlane) and are tolerated; profiles/archive/r01_kernel_resources.txt
    # lists them.
    bad = [n for n, r in recs.items() if r.get("private_segment_fixed_size", 0) or r.get("vgpr_spill_count", 0)]
    assert not bad, bad


def _blocks_per_cu(r):
    # a block of B threads spreads B / 256 waves over each of the 4 SIMDs
    per_simd = max(1, r.get("max_flat_workgroup_size", 256) // 256)
    return r["waves_per_simd"] // per_simd


def test_lds_never_limits_occupancy(recs):
    # 160 KiB LDS per CU. A kernel with W waves per SIMD and blocks of B threads keeps W * 256 / B
    # blocks resident per CU (W for the 256-thread blocks most kernels use): their LDS must fit next
    # to each other, so LDS never becomes the occupancy limiter (the VGPR budget is). The streaming
    # K-step kernel (heat7_tbk: LDS-DMA planes + seam tables, up to 49 KiB at one wave per SIMD)
    # is the largest user.
    bad = {n: (r.get("group_segment_fixed_size", 0), r["waves_per_simd"]) for n, r in recs.items()
           if _blocks_per_cu(r) < 1 or r.get("group_segment_fixed_size", 0) * _blocks_per_cu(r) > 160 * 1024}
    assert not bad, bad


@pytest.mark.parametrize("name,min_waves", [
    # the shipped headline sweep: 1024^3 fp32, 4 fused steps, 3 + 2-row bands of 8 waves (one 512-thread
    # block per CU: 2 waves per SIMD is all a block of 8 waves can have)
    ("mdfx::dev::heat7_wxk<float, 3, 2, 4, 8, false, false, false, 0>", 2),
    ("mdfx::dev::heat7_wxk<float, 3, 2, 4, 8, false, true, false, 0>", 2),   # its pencil copy
    ("mdfx::dev::heat7_wxk<float, 3, 2, 4, 8, false, false, true, 0>", 2),   # folded-boundary copy (N > 1)
    ("mdfx::dev::heat7_wxk<float, 2, 2, 4, 2, false, true, false, 0>", 2),   # pencil y strips (2-wave bands)
    ("mdfx::dev::heat7_wxk<float, 3, 2, 4, 8, true, false, true, 0>", 2),
    ("mdfx::dev::heat7_wxk<float, 3, 2, 4, 8, true, false, false, 0>", 2),         # its residual sweeps
    ("mdfx::dev::heat7_wxk<float, 5, 4, 5, 8, false, false, false, 2>", 2),        # fp32 K = 5 (2-cell lanes): the default
    ("mdfx::dev::heat7_wxk<float, 5, 4, 5, 8, true, false, false, 2>", 2),
    ("mdfx::dev::heat7_wxk<float, 5, 4, 5, 8, false, false, true, 2>", 2),         # its folded-boundary copy
    ("mdfx::dev::heat7_wxk<float, 5, 4, 5, 8, true, false, true, 2>", 2),
    ("mdfx::dev::heat7_wxk<float, 4, 4, 3, 8, false, false, false, 0>", 2),        # K = 3 (step-count remainders)
    ("mdfx::dev::heat7_wxk<double, 3, 1, 3, 8, false, false, false, 0>", 2),       # fp64 K = 3 (2048^3 + residual)
    ("mdfx::dev::heat7_wxk<double, 3, 1, 3, 8, true, false, false, 0>", 2),
    ("mdfx::dev::heat7_wxk<double, 2, 1, 4, 8, false, false, false, 0>", 2),       # fp64 K = 4 (the default from 1024-cell rows)
    ("mdfx::dev::heat7_wxk<double, 2, 1, 4, 8, true, false, false, 0>", 2),
    ("mdfx::dev::heat7_wxk<double, 2, 1, 4, 8, false, false, true, 0>", 2),        # its folded-boundary copy
    ("mdfx::dev::heat7_wxk<double, 5, 4, 5, 8, false, false, false, 1>", 2),       # fp64 K = 5 (1-cell lanes)
    ("mdfx::dev::heat7_wxk<double, 5, 4, 5, 8, true, false, false, 1>", 2),
    ("mdfx::dev::heat7_wxk<double, 5, 4, 5, 8, false, false, true, 1>", 2),        # its folded-boundary copy
    ("mdfx::dev::box27_wxk<float, 2, 1, 3, 8, false, 0, 2>", 4),       # 27-point K = 3 fp32 rows > 512: 2-cell lanes, 2 bands per CU
    ("mdfx::dev::box27_wxk<float, 2, 1, 3, 8, true, 0, 2>", 3),
    ("mdfx::dev::box27_wxk<float, 2, 1, 3, 4, false, 2, 0>", 2),       # fp32 rows <= 512: whole-row blocks
    ("mdfx::dev::box27_wxk<float, 2, 1, 3, 4, true, 2, 0>", 2),
    ("mdfx::dev::box27_wxk<double, 2, 1, 3, 8, false, 0, 0>", 2),
    ("mdfx::dev::box27_wxk<double, 2, 1, 3, 8, true, 0, 0>", 2),
    ("mdfx::dev::box27_tb2n<1, 1, false>", 3),                          # 27-point K = 2 fp32 (512^3)
    ("mdfx::dev::heat7_wtk<double, 2, 3, 8, false, 0>", 2),
    ("mdfx::dev::jacobi5_tbk<float, 8, false, false, 2>", 3),           # 2D MDF, 8 steps per sweep
    ("mdfx::dev::jacobi5_tbk<float, 8, false, true, 1>", 4),            # reference precision (no unroll)
    ("mdfx::dev::heat7_tbk<float, 4, 2, 4, false>", 2),                 # K = 2 fused sweep
    ("mdfx::dev::heat7_tbk<double, 4, 2, 4, false>", 2),
    ("mdfx::dev::heat7_tb2<float, 2, 4, false, 1, true>", 3),           # x-tiled rows
    ("mdfx::dev::heat7_tb2<double, 2, 4, false, 1, true>", 3),
    ("mdfx::dev::heat7_zw<float, 2, 4, false, false, 1>", 6),           # single-step default
    ("mdfx::dev::box27_zw<float, 2, 4, false>", 4),
])
def test_default_kernels_keep_their_occupancy(recs, name, min_waves):
    assert name in recs, sorted(k for k in recs if name.split("<")[0] in k)[:8]
    assert recs[name]["waves_per_simd"] >= min_waves, recs[name]


def test_headline_sweep_keeps_its_memory_waits():
    # the 1024^3 slab sweep (heat7_wxk fp32 K = 4) waits for ALL outstanding vector-memory ops in
    # 13 places; round 4's pencil row bounds, compiled into the same kernel, made it 19 (six waits in
    # front of window LDS reads: the sweep lost 3-4 %, profiles/r04_session_c/summary.txt). The
    # slab and pencil copies are separate instances now: pin the slab one's count.
    isa = kernel_isa(LIB, "_ZN4mdfx3dev9heat7_wxkIfLi3ELi2ELi4ELi8ELb0ELb0ELb0ELi0E")
    assert len(isa) == 1, sorted(isa)
    body = next(iter(isa.values()))
    assert len(body) > 5000
    n0 = sum(1 for l in body if l.startswith("s_waitcnt") and "vmcnt(0)" in l)
    assert n0 <= 13, n0


def test_k5_sweep_keeps_its_memory_waits():
    # the fp32 K = 5 sweep (2-cell lanes, 4-byte window DMAs) and its folded-boundary copy: the same
    # 13 full vector-memory waits as the K = 4 sweep (none in front of the window reads)
    for mangled in ("_ZN4mdfx3dev9heat7_wxkIfLi5ELi4ELi5ELi8ELb0ELb0ELb0ELi2E",
                    "_ZN4mdfx3dev9heat7_wxkIfLi5ELi4ELi5ELi8ELb0ELb0ELb1ELi2E"):
        isa = kernel_isa(LIB, mangled)
        assert len(isa) == 1, sorted(isa)
        body = next(iter(isa.values()))
        n0 = sum(1 for l in body if l.startswith("s_waitcnt") and "vmcnt(0)" in l)
        assert n0 <= 13, (mangled, n0)


def test_folded_boundary_copy_keeps_the_sweep_loop():
    # the folded-boundary copy adds one out-of-line signal call; its plane loop must keep the same
    # memory waits as the plain sweep (13 vmcnt(0))
    isa = kernel_isa(LIB, "_ZN4mdfx3dev9heat7_wxkIfLi3ELi2ELi4ELi8ELb0ELb0ELb1ELi0E")
    assert len(isa) == 1, sorted(isa)
    body = next(iter(isa.values()))
    n0 = sum(1 for l in body if l.startswith("s_waitcnt") and "vmcnt(0)" in l)
    assert n0 <= 13, n0

"""CPU tier (T1 of SURVEY §4.3): slab math, CPU oracle vs PyTorch, engine invariants.

The native engine runs the same scheduler on the CPU backend (host transport), so decomposition
invariance, overlap/serialised equivalence, residuals and checkpoint re-decomposition are all
covered here without a GPU.
"""

import json
import os

import numpy as np
import pytest
import torch

import mpi_cuda_process_amd as m
from mpi_cuda_process_amd.ops import (FieldLayout, alloc_field, apply_stencil, init_field, reference)
from mpi_cuda_process_amd.parallel.decomp import neighbors, owner, slab_bounds


# ---- slab decomposition --------------------------------------------------------------------
@pytest.mark.parametrize("nz,parts", [(10, 1), (10, 3), (7, 7), (1024, 8), (1025, 8), (13, 4)])
def test_slab_bounds_cover_and_match_native(mdfx, nz, parts):
    b = slab_bounds(nz, parts)
    assert b[0][0] == 0 and b[-1][1] == nz
    assert all(b[i][1] == b[i + 1][0] for i in range(parts - 1))
    sizes = [e - s for s, e in b]
    assert max(sizes) - min(sizes) <= 1
    assert [tuple(x) for x in mdfx.native().slab_bounds(nz, parts)] == b
    for z in range(nz):
        p = owner(z, nz, parts)
        assert b[p][0] <= z < b[p][1]


def test_slab_bounds_errors():
    with pytest.raises(ValueError):
        slab_bounds(3, 4)
    with pytest.raises(ValueError):
        slab_bounds(3, 0)
    assert neighbors(0, 3) == (-1, 1) and neighbors(2, 3) == (1, -1)


def test_layout_pitch_alignment(mdfx):
    for dt, es in (("f32", 4), ("f64", 8), ("u8", 1)):
        d = mdfx.native().layout(100, 3, 10, 2, 5, 1, dt)
        assert d["pitch"] * es % 256 == 0 and d["pitch"] >= 100
        assert d["planes"] == 3 + 2 and d["plane"] == d["pitch"] * 3


# ---- CPU oracle kernels vs plain PyTorch -----------------------------------------------------
PROBS = [m.heat3d(nx=23, ny=17, nz=13), m.heat3d(nx=19, ny=11, nz=9, dtype="f64"),
         m.box27(nx=21, ny=15, nz=11), m.box27(nx=12, ny=9, nz=8, dtype="f64"), m.mdf2d(h=29, w=31),
         m.mdf2d(h=17, w=40, dtype="f64"), m.life2d(h=33, w=41)]


def _ids(p):
    return p.describe().replace(" ", "_")


@pytest.mark.parametrize("prob", PROBS, ids=_ids)
def test_cpu_kernel_vs_torch_reference(mdfx, prob):
    lay = FieldLayout.make(prob)
    a, b = alloc_field(lay), alloc_field(lay)
    init_field(prob, lay, a)
    apply_stencil(prob, lay, a, b)
    u = a[lay.owned, :, : lay.nx]
    got = b[lay.owned, :, : lay.nx]
    ref = reference.step(prob.kind, u.double() if prob.dtype != "u8" else u, **prob.coef_kwargs())
    if prob.dtype == "u8":
        assert torch.equal(got, ref)
    else:
        assert (got.double() - ref).abs().max().item() < (2e-6 if prob.dtype == "f32" else 1e-13)


def test_dirichlet_boundary_held(mdfx):
    prob = m.mdf2d(h=16, w=16)
    with m.Simulation(prob, device="cpu", ranks=2) as sim:
        sim.init()
        sim.run(25)
        g = sim.gather()[:, 0, :]
    assert (g[0] == 100).all() and (g[-1] == 100).all() and (g[:, 0] == 100).all() and (g[:, -1] == 100).all()
    assert 0 < g[8, 8] < 100  # heat diffused into the interior (the reference never advanced: D1)


def test_mdf_matches_reference_formula(mdfx):
    """u' = u + 0.25 (E + W + N + S - 4u) with edges 100 / interior 0 (MDF_kernel.cu:20, :88-99)."""
    prob = m.mdf2d(h=9, w=11)
    with m.Simulation(prob, device="cpu") as sim:
        sim.init()
        u = sim.gather()[:, 0, :].astype(np.float64)
        sim.run(1)
        got = sim.gather()[:, 0, :]
    want = u.copy()
    want[1:-1, 1:-1] = u[1:-1, 1:-1] + 0.25 * (u[1:-1, 2:] + u[1:-1, :-2] + u[:-2, 1:-1] + u[2:, 1:-1]
                                               - 4 * u[1:-1, 1:-1])
    assert np.abs(got - want).max() < 1e-4


def test_life_blinker_and_glider(mdfx):
    prob = m.life2d(h=12, w=12)
    board = np.zeros((12, 1, 12), np.uint8)
    board[5, 0, 4:7] = 1  # blinker
    with m.Simulation(prob, device="cpu", ranks=3) as sim:
        sim.init(m.InitCondition(kind="constant", value=0))
        for i in range(3):
            lay = sim.layout(i)
            sim.write_local(i, board[lay["z0"]:lay["z1"]])
        sim.run(1)
        g = sim.gather()[:, 0, :]
        assert g[4:7, 5].tolist() == [1, 1, 1] and g.sum() == 3
        sim.run(1)
        g = sim.gather()[:, 0, :]
        assert g[5, 4:7].tolist() == [1, 1, 1] and g.sum() == 3


def test_life_compat_init_is_glibc_rand(mdfx):
    import ctypes

    libc = ctypes.CDLL("libc.so.6")
    libc.srand(1)
    h, w = 6, 7
    want = np.zeros((h, w), np.uint8)
    for i in range(h):
        for j in range(w):
            if i in (0, h - 1) or j in (0, w - 1):
                continue
            rp = np.float32(libc.rand()) / np.float32(2147483647)
            want[i, j] = 0 if rp > np.float32(0.15) else 1
    got = mdfx.native().life_compat_init(h, w, 0.15, 1)
    assert np.array_equal(got, want)


# ---- engine invariants on the CPU backend ----------------------------------------------------
@pytest.mark.parametrize("prob", PROBS, ids=_ids)
def test_decomposition_invariance_cpu(mdfx, prob):
    def run(p):
        with m.Simulation(prob, device="cpu", ranks=p) as sim:
            sim.init()
            sim.run(5)
            return sim.gather()

    base = run(1)
    for p in (2, 3, min(5, prob.nz)):
        assert np.array_equal(base, run(p)), p


def test_overlap_flag_and_sync_debug_equivalent(mdfx):
    prob = m.heat3d(nx=20, ny=10, nz=12)
    outs = []
    for kw in (dict(overlap=True), dict(overlap=False), dict(sync_debug=True)):
        with m.Simulation(prob, device="cpu", ranks=4, **kw) as sim:
            sim.init()
            sim.run(6)
            outs.append(sim.gather())
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])


def test_residual_cpu(mdfx):
    prob = m.heat3d(nx=16, ny=12, nz=10)
    with m.Simulation(prob, device="cpu", ranks=2, residual_every=2) as sim:
        sim.init()
        sim.run(1)
        assert sim.residual < 0
        a = sim.gather()
        sim.run(1)
        b = sim.gather()
        assert sim.native.residual_step == 2
        want = float(np.sqrt(((b.astype(np.float64) - a) ** 2).sum()))
        assert abs(sim.residual - want) < 1e-9 * max(1, want)


def test_residual_decreases_for_jacobi(mdfx):
    prob = m.mdf2d(h=32, w=32)
    with m.Simulation(prob, device="cpu", residual_every=10) as sim:
        sim.init()
        res = []
        for _ in range(5):
            sim.run(10)
            res.append(sim.residual)
    assert all(res[i + 1] < res[i] for i in range(4))


def test_divergence_raises(mdfx):
    prob = m.heat3d(nx=12, ny=12, nz=12, r=10.0)  # unstable explicit step
    with m.Simulation(prob, device="cpu", residual_every=5) as sim:
        sim.init(m.InitCondition(kind="random", lo=-1e30, hi=1e30))
        with pytest.raises(RuntimeError, match="non-finite"):
            sim.run(400)


def test_checkpoint_roundtrip_redecompose(mdfx, tmp_path):
    prob = m.box27(nx=14, ny=9, nz=15)
    with m.Simulation(prob, device="cpu", ranks=1) as sim:
        sim.init()
        sim.run(7)
        ref = sim.gather()
    with m.Simulation(prob, device="cpu", ranks=3) as sim:
        sim.init()
        sim.run(4)
        sim.save_checkpoint(str(tmp_path / "ck"))
    hdr = json.load(open(os.path.join(tmp_path, "ck", "slab_1.json")))
    assert hdr["step"] == 4 and hdr["nranks"] == 3 and hdr["format"] == "mdfx-slab-v1"
    with m.Simulation(prob, device="cpu", ranks=4) as sim:
        sim.load_checkpoint(str(tmp_path / "ck"))
        sim.run(3)
        assert np.array_equal(ref, sim.gather())


def test_checkpoint_mismatch_rejected(mdfx, tmp_path):
    with m.Simulation(m.heat3d(n=8), device="cpu") as sim:
        sim.init()
        sim.save_checkpoint(str(tmp_path / "ck"))
    with m.Simulation(m.heat3d(n=9), device="cpu") as sim:
        with pytest.raises(RuntimeError, match="does not match"):
            sim.load_checkpoint(str(tmp_path / "ck"))


def test_write_owned_refreshes_ghosts(mdfx):
    prob = m.heat3d(nx=10, ny=8, nz=9)
    rng = np.random.default_rng(0)
    u = rng.random((9, 8, 10), dtype=np.float32)
    with m.Simulation(prob, device="cpu", ranks=3) as sim:
        sim.init(m.InitCondition(kind="constant", value=0))
        for i in range(3):
            lay = sim.layout(i)
            sim.write_local(i, u[lay["z0"]:lay["z1"]])
        sim.run(2)
        got = sim.gather()
    ref = reference.run("heat7", torch.from_numpy(u).double(), 2).numpy()
    assert np.abs(got - ref).max() < 1e-5


def test_bad_configs_rejected(mdfx):
    with pytest.raises(ValueError):
        m.Problem("life", 8, 1, 8, dtype="f32")
    with pytest.raises(ValueError):
        m.Problem("heat7", 8, 8, 8, dtype="u8")
    with pytest.raises(RuntimeError):
        m.Simulation(m.heat3d(n=4), device="cpu", ranks=5)  # more ranks than planes


def test_kernel_region_outside_owned_rejected(mdfx):
    prob = m.heat3d(nx=8, ny=8, nz=8)
    lay = FieldLayout.make(prob)
    a, b = alloc_field(lay), alloc_field(lay)
    with pytest.raises(ValueError):
        apply_stencil(prob, lay, a, b, 0, 3)


# ---- temporal blocking (2 fused steps per sweep, halo 2) ----------------------------------------
@pytest.mark.parametrize("ranks", [1, 2, 3, 5])
@pytest.mark.parametrize("steps", [1, 2, 7, 10])
def test_temporal2_equals_single_steps_cpu(mdfx, ranks, steps):
    prob = m.heat3d(nx=14, ny=11, nz=13)
    with m.Simulation(prob, device="cpu") as sim:
        sim.init()
        sim.run(steps)
        ref = sim.gather()
    with m.Simulation(prob, device="cpu", ranks=ranks, temporal=2) as sim:
        assert sim.temporal == 2 and sim.layout(0)["halo"] == 2
        sim.init()
        sim.run(steps)
        assert sim.steps == steps
        assert np.array_equal(ref, sim.gather())


@pytest.mark.parametrize("every", [1, 2, 3, 4])
def test_temporal2_residual_schedule(mdfx, every):
    prob = m.heat3d(nx=12, ny=10, nz=11)
    res = {}
    for t in (1, 2):
        with m.Simulation(prob, device="cpu", ranks=2, temporal=t, residual_every=every) as sim:
            sim.init()
            sim.run(9)
            res[t] = (sim.residual, sim.native.residual_step, sim.gather())
    assert res[1][1] == res[2][1] == (9 // every) * every
    assert abs(res[1][0] - res[2][0]) <= 1e-9 * max(1.0, res[1][0])
    assert np.array_equal(res[1][2], res[2][2])


def test_temporal2_checkpoint_roundtrip(mdfx, tmp_path):
    prob = m.heat3d(nx=12, ny=9, nz=16)
    with m.Simulation(prob, device="cpu") as sim:
        sim.init()
        sim.run(9)
        ref = sim.gather()
    with m.Simulation(prob, device="cpu", ranks=3, temporal=2) as sim:
        sim.init()
        sim.run(4)
        sim.save_checkpoint(str(tmp_path / "ck"))
    with m.Simulation(prob, device="cpu", ranks=2, temporal=2) as sim:
        sim.load_checkpoint(str(tmp_path / "ck"))
        sim.run(5)
        assert np.array_equal(ref, sim.gather())


def test_temporal_depth_validated(mdfx):
    with pytest.raises(RuntimeError):
        m.Simulation(m.heat3d(n=8), device="cpu", temporal=17)  # 1..16 (16: the bit-sliced Life)
    with pytest.raises(RuntimeError, match="ghost planes"):  # slabs thinner than the exchanged halo
        m.Simulation(m.mdf2d(h=20, w=16), device="cpu", ranks=4, temporal=8)


@pytest.mark.parametrize("temporal", [3, 4, 8])
@pytest.mark.parametrize("prob", [m.mdf2d(h=61, w=37), m.life2d(h=70, w=45)], ids=["mdf", "life"])
def test_deep_temporal_2d_equals_single_steps_cpu(mdfx, prob, temporal):
    """Deep temporal blocking (halo = K rows, K fused steps per sweep) of the 2D problems, with
    residual evaluations that fall inside and between sweeps."""
    with m.Simulation(prob, device="cpu", residual_every=5) as sim:
        sim.init()
        sim.run(23)
        ref, rr = sim.gather(), sim.residual
    with m.Simulation(prob, device="cpu", ranks=3, temporal=temporal, residual_every=5) as sim:
        assert sim.layout(0)["halo"] == temporal
        sim.init()
        sim.run(23)
        assert sim.steps == 23
        assert np.array_equal(ref, sim.gather()) and abs(sim.residual - rr) <= 1e-9 * max(1.0, rr)


def test_sweep_plan(mdfx):
    """run() cuts every stretch up to a residual step into sweeps of the deepest depth and a
    remainder of the deepest depth that fits (the residual sweep last); sweep_plan() reports the
    sweeps a run would issue, and the result equals single steps bitwise."""
    prob = m.heat3d(nx=40, ny=24, nz=36)
    with m.Simulation(prob, device="cpu", ranks=2, temporal=4, residual_every=10) as sim:
        assert sim.sweep_plan(20) == [(4, False), (4, False), (2, True)] * 2
        assert sim.sweep_plan(12) == [(4, False), (4, False), (2, True), (2, False)]
        sim.init()
        sim.run(5)
        assert sim.steps == 5 and sim.sweep_plan(5) == [(4, False), (1, True)]
        assert sim.sweep_plan(17) == [(4, False), (1, True), (4, False), (4, False), (2, True), (2, False)]
        sim.run(17)
        got, gr = sim.gather(), sim.residual
    with m.Simulation(prob, device="cpu", temporal=4) as sim:
        assert sim.sweep_plan(9) == [(4, False), (4, False), (1, False)]
    with m.Simulation(prob, device="cpu", residual_every=10) as sim:
        assert sim.sweep_plan(3) == [(1, False)] * 3
        sim.init()
        sim.run(22)
        assert np.array_equal(got, sim.gather()) and abs(gr - sim.residual) <= 1e-12 * max(1.0, gr)


def test_sweep_plan_cost_tables(mdfx):
    """The planner with the GPU's cost tables (hip_sweep_cost, host-side): on 1024-cell 7-point rows
    a 10-step residual stretch at depth 4 runs 4 + 3 + 3 (the two-step kernels are the least
    efficient per step), at depth 3 in fp64 3 + 3 + 3 + 1 (the single step runs near the copy roof;
    the measured order, profiles/r04_session_n/); other stencils keep the deepest sweeps first; a
    missing depth (pencils have no two-step kernel) is planned around; the residual sweep is last."""
    import mpi_cuda_process_amd as m

    n = m.native()

    def plan(steps, every, T, kind="heat7", dtype="f32", nx=1024, start=0, missing=()):
        cost = [0.0] + [n.hip_sweep_cost(kind, dtype, nx, k) for k in range(1, 17)]
        ok = [False] + [k not in missing for k in range(1, 17)]
        return [tuple(x) for x in n.plan_sweeps(steps, start, every, T, cost, ok)]

    F, R = False, True
    for dt in ("f32", "f64"):
        assert plan(10, 10, 4, dtype=dt) == [(4, F), (3, F), (3, R)]
        assert plan(12, 12, 4, dtype=dt) == [(4, F), (4, F), (4, R)]
        assert plan(20, 0, 4, dtype=dt) == [(4, F)] * 5
    assert plan(10, 10, 3, dtype="f64") == [(3, F), (3, F), (3, F), (1, R)]
    assert plan(5, 0, 4, dtype="f64") == [(4, F), (1, F)]
    assert plan(10, 10, 4, kind="box27", nx=512) == [(4, F), (4, F), (2, R)]    # generic costs
    assert plan(6, 0, 4, missing=(2,)) == [(3, F), (3, F)]                      # no 2-step kernel
    assert plan(2, 0, 4, missing=(2, 3)) == [(1, F), (1, F)]
    assert plan(17, 10, 4, start=5) == [(3, F), (2, R), (4, F), (3, F), (3, R), (2, F)]  # fp32: 3 + 2 < 4 + 1
    assert plan(7, 0, 1) == [(1, F)] * 7


def test_cpu_avx2_and_baseline_builds_bitwise_equal(tmp_path):
    """The CPU stencils exist twice (baseline x86-64 with libm's software fma, and AVX2 + FMA chosen
    at run time); both are exact, so every stencil must agree bit for bit."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import numpy as np, mpi_cuda_process_amd as m\n"
            "out = {}\n"
            "for name, prob in [('h', m.heat3d(nx=37, ny=21, nz=19)), ('b', m.box27(nx=29, ny=17, nz=13, dtype='f64')),\n"
            "                   ('j', m.mdf2d(h=77, w=91)), ('l', m.life2d(h=60, w=70))]:\n"
            "    with m.Simulation(prob, device='cpu', ranks=2, residual_every=3) as sim:\n"
            "        sim.init(); sim.run(7); out[name] = sim.gather(); out[name + 'r'] = np.array(sim.residual)\n"
            "np.savez(sys.argv[1], **out)\n") % root
    res = {}
    for tag, env in (("avx2", {}), ("base", {"MDFX_CPU_BASELINE": "1"})):
        f = str(tmp_path / (tag + ".npz"))
        p = subprocess.run([sys.executable, "-c", code, f], env=dict(os.environ, OMP_NUM_THREADS="2", **env),
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)
        assert p.returncode == 0, p.stderr.decode()[-2000:]
        res[tag] = np.load(f)
    for k in res["avx2"].files:
        assert np.array_equal(res["avx2"][k], res["base"][k]), k


@pytest.mark.parametrize("prob,steps,temporal", [(m.heat3d(nx=20, ny=9, nz=11), 7, 0), (m.heat3d(nx=20, ny=9, nz=11), 7, 2),
                                                 (m.mdf2d(h=30, w=17), 9, 4), (m.life2d(h=40, w=33), 6, 3),
                                                 (m.box27(nx=13, ny=12, nz=10, dtype="f64"), 5, 2)])
def test_advance_functional_api(mdfx, prob, steps, temporal):
    with m.Simulation(prob, device="cpu") as sim:
        sim.init()
        g0 = torch.from_numpy(sim.gather().copy())
        sim.run(steps)
        ref = sim.gather()
    out = m.advance(prob, g0, steps, temporal=temporal)
    assert np.array_equal(out.numpy(), ref)
    if prob.ny == 1:  # 2D grids may be passed as (h, w)
        assert np.array_equal(m.advance(prob, g0.squeeze(1), steps, temporal=temporal).numpy(), ref.squeeze(1))


def test_auto_temporal_rule(mdfx):
    from mpi_cuda_process_amd.engine import auto_temporal

    assert auto_temporal(m.heat3d(n=64), 1, "cpu") == 1
    with m.Simulation(m.mdf2d(h=64, w=32), device="cpu", temporal=0) as sim:
        assert sim.temporal == 1  # the CPU never fuses by default


def test_checkpoint_stale_slabs_ignored(mdfx, tmp_path):
    """Saving with 4 ranks, then with 2 ranks into the same directory: both readers return the
    2-rank state (the extra slab_2 / slab_3 files are removed, and readers trust slab_0's nranks)."""
    import mpi_cuda_process_amd as m
    from mpi_cuda_process_amd.utils.checkpoint import read_checkpoint

    prob = m.heat3d(nx=12, ny=9, nz=16)
    d = str(tmp_path / "ck")
    with m.Simulation(prob, device="cpu", ranks=4) as s4:
        s4.init()
        s4.run(1)
        s4.save_checkpoint(d)
    with m.Simulation(prob, device="cpu", ranks=2) as s2:
        s2.init()
        s2.run(5)
        want = s2.gather()
        s2.save_checkpoint(d)
    assert sorted(f for f in os.listdir(d) if f.endswith(".json")) == ["slab_0.json", "slab_1.json"]
    grid, metas = read_checkpoint(d)
    assert np.array_equal(grid, want) and {mm["step"] for mm in metas} == {5}
    with m.Simulation(prob, device="cpu", ranks=3) as s3:
        s3.load_checkpoint(d)
        assert np.array_equal(s3.gather(), want) and s3.steps == 5


def test_checkpoint_mixed_steps_rejected(mdfx, tmp_path):
    import json as _json

    import mpi_cuda_process_amd as m

    prob = m.heat3d(nx=10, ny=8, nz=12)
    d = str(tmp_path / "ck")
    with m.Simulation(prob, device="cpu", ranks=2) as s:
        s.init()
        s.run(2)
        s.save_checkpoint(d)
    h = _json.load(open(os.path.join(d, "slab_1.json")))
    h["step"] = 7
    _json.dump(h, open(os.path.join(d, "slab_1.json"), "w"))
    with m.Simulation(prob, device="cpu", ranks=2) as s:
        with pytest.raises(RuntimeError, match="does not match slab_0"):
            s.load_checkpoint(d)


def test_graph_request_with_host_transport_runs_eagerly(mdfx):
    """graph=True with a transport whose exchange moves data on the host falls back to eager steps
    (same result as graph=False)."""
    import mpi_cuda_process_amd as m

    prob = m.heat3d(nx=14, ny=10, nz=12)
    outs = []
    for g in (False, True):
        with m.Simulation(prob, device="cpu", ranks=3, graph=g) as s:
            s.init()
            s.run(6)
            outs.append(s.gather())
    assert np.array_equal(outs[0], outs[1])


def _reference_mdf_numpy(g, steps):
    """The reference's MDF update (MDF_kernel.cu:20) emulated in numpy: fp32 sum ((E+W)+N)+S, the
    contracted fmaf(-4, C, sum) (exact in fp64, then one rounding to fp32), then 0.25*t + C in fp64
    (0.25*t is exact) rounded to fp32 at the store; boundary cells held."""
    u = g.astype(np.float32)
    for _ in range(steps):
        c = u[1:-1, 1:-1]
        s = ((u[1:-1, 2:] + u[1:-1, :-2]) + u[:-2, 1:-1]) + u[2:, 1:-1]  # fp32 adds
        t = (np.float64(-4.0) * c.astype(np.float64) + s.astype(np.float64)).astype(np.float32)
        v = (np.float64(0.25) * t.astype(np.float64) + c.astype(np.float64)).astype(np.float32)
        n = u.copy()
        n[1:-1, 1:-1] = v
        u = n
    return u


@pytest.mark.parametrize("ranks", [1, 3])
def test_mdf_ref_precision_matches_reference_arithmetic(mdfx, ranks):
    """mdf2d(ref_precision=True) reproduces the reference's mixed fp32/fp64 update bit for bit
    (random data, so the rounding differences from the all-fp32 update actually occur)."""
    import mpi_cuda_process_amd as m

    prob = m.mdf2d(h=37, w=53, ref_precision=True).with_init(kind="random", seed=3, lo=-50.0, hi=150.0)
    with m.Simulation(prob, device="cpu", ranks=ranks) as sim:
        sim.init()
        g0 = sim.gather()[:, 0, :]
        sim.run(7)
        got = sim.gather()[:, 0, :]
    want = _reference_mdf_numpy(g0, 7)
    assert np.array_equal(got, want)
    plain = m.mdf2d(h=37, w=53).with_init(kind="random", seed=3, lo=-50.0, hi=150.0)
    with m.Simulation(plain, device="cpu") as sim:
        sim.init()
        sim.run(7)
        other = sim.gather()[:, 0, :]
    assert np.abs(other - want).max() < 1e-3  # same update up to rounding


def test_mdf_ref_precision_runs_fused(mdfx):
    """The reference's mixed-precision MDF update has fused kernels (jacobi5_tbk REF), so the
    reference-compatible dialogue gets the deep temporal blocking too."""
    import mpi_cuda_process_amd as m

    for k in (2, 3, 4, 6, 8):
        assert m.native().hip_supports_steps("jacobi5", "f32", 64, 1, 64, k, k, True)
    from mpi_cuda_process_amd.engine import auto_temporal

    assert auto_temporal(m.mdf2d(h=4096, w=512, ref_precision=True), 1, "hip") == 8
    assert auto_temporal(m.mdf2d(h=4096, w=512), 1, "hip") == 8


@pytest.mark.parametrize("r", [0.25, 0.5, 0.125])
def test_mdf_ref_precision_at_power_of_two_rate_is_bitwise_fp32(mdfx, r):
    """StencilSpec::mixed_update: with a power-of-two r the reference's round_f32(round_f64(r*t + u))
    equals fma_f32(r, t, u) for every input, so ref_precision and the plain update agree bit for
    bit (the CPU oracle evaluates both literally; values spanning 2^-30..2^30 exercise wide
    exponent gaps, where fp64 itself rounds)."""
    import mpi_cuda_process_amd as m

    out = []
    for ref in (False, True):
        prob = m.mdf2d(h=41, w=67, r=r, ref_precision=ref).with_init(kind="random", seed=11, lo=-50.0, hi=150.0)
        with m.Simulation(prob, device="cpu") as sim:
            sim.init()
            g = sim.gather()
            g[:, 0, :] *= np.exp2(np.random.default_rng(3).integers(-30, 30, g[:, 0, :].shape)).astype(np.float32)
            sim.write_local(0, g)
            sim.run(5)
            out.append(sim.gather())
    assert np.array_equal(out[0], out[1])


def test_fused_depth_policy(mdfx):
    """hip_fused_depth: the measured-win fused depth per stencil and row width (host-side policy,
    profiles/archive/r02_wtk/README.txt, r03_wtk/, r03_wxk/): for the 3D 7-point where the x segments cover
    at least 2/3 of the lane cells (rows of 512 cells and more) K = 5 through heat7_wxk in fp32
    (2-cell lanes), in fp64 K = 5 from rows of 2048 cells (1-cell lanes, round 6) and K = 4 below, 2
    below 512; the 27-point 3 (box27_wxk) in fp64, at fp32 rows of 257..512 cells (whole-row
    blocks) and of 1024 cells and more, else 2;
    8 / 12 for the 2D stencils; auto_temporal makes it shallower for thin slabs (5 -> 4 -> 2 -> 1,
    3 -> 2 -> 1)."""
    import mpi_cuda_process_amd as m
    from mpi_cuda_process_amd.engine import auto_temporal

    d = m.native().hip_fused_depth
    assert d("heat7", "f32", 1024) == 5 and d("heat7", "f64", 1024) == 4
    assert d("heat7", "f32", 2048) == 5 and d("heat7", "f64", 2048) == 5 and d("heat7", "f32", 3072) == 5
    assert d("heat7", "f64", 2047) == 4 and d("heat7", "f64", 4096) == 5
    # the sweep plan's cost of an fp64 5-step sweep follows the row width it is the default for
    c = m.native().hip_sweep_cost
    assert c("heat7", "f64", 2048, 5) < c("heat7", "f64", 1024, 5)
    assert auto_temporal(m.heat3d(n=2048, dtype="f64"), 8, "hip") == 5   # config 5: 256-plane slabs
    assert d("heat7", "f32", 512) == 5 and d("heat7", "f32", 256) == 2 and d("heat7", "f64", 512) == 4
    assert d("box27", "f32", 512) == 3 and d("box27", "f32", 1024) == 3 and d("box27", "f64", 512) == 3
    assert d("box27", "f32", 256) == 2 and d("box27", "f32", 768) == 2
    assert d("jacobi5", "f32", 16384) == 8 and d("life", "u8", 32768) == 12
    assert auto_temporal(m.heat3d(n=1024), 8, "hip") == 5       # 128-plane slabs: 5 steps per sweep
    assert auto_temporal(m.heat3d(nx=1024, ny=64, nz=152), 8, "hip") == 4   # 19-plane slabs: 5 -> 4
    assert auto_temporal(m.heat3d(n=1024, dtype="f64"), 8, "hip") == 4
    assert auto_temporal(m.heat3d(n=512, dtype="f64"), 8, "hip") == 4
    assert auto_temporal(m.heat3d(nx=1024, ny=64, nz=64), 8, "hip") == 2   # 8-plane slabs
    assert auto_temporal(m.heat3d(nx=1024, ny=64, nz=24), 8, "hip") == 1
    assert auto_temporal(m.heat3d(n=1024), 1, "cpu") == 1


def test_interval_depth_follows_the_residual_interval(mdfx):
    """The auto depth follows the residual interval (round 6, 2048^3 fp64, a residual every 12
    steps): on one GPU depth 5's plan 5 + 4 + 3 (measured 1022 GCells/s) beats depth 4's 4 + 4 + 4
    (961-985); with several ranks every sweep exchanges and recomputes halo-deep boundary regions, so
    depth 4's whole 4-step sweeps win (N = 8 rank proxy 878-880 vs 841-849). Intervals that are
    whole 5-step sweeps keep depth 5 either way."""
    import mpi_cuda_process_amd as m
    from mpi_cuda_process_amd.engine import auto_temporal

    nat = m.native()
    c = [0.0] + [nat.hip_sweep_cost("heat7", "f64", 2048, k) for k in range(1, 6)]
    ok = [False] + [True] * 5
    assert [k for k, _ in nat.plan_sweeps(12, 0, 12, 5, c, ok)] == [5, 4, 3]
    assert [k for k, _ in nat.plan_sweeps(12, 0, 12, 4, c, ok)] == [4, 4, 4]
    assert nat.interval_depth(12, 5, c, ok) == 5 and nat.interval_depth(12, 5, c, ok, True) == 4
    for uniform in (False, True):
        assert nat.interval_depth(10, 5, c, ok, uniform) == 5 and nat.interval_depth(20, 5, c, ok, uniform) == 5
        assert nat.interval_depth(0, 5, c, ok, uniform) == 5 and nat.interval_depth(7, 1, c, ok, uniform) == 1
    # a depth whose interval plan never runs it is never chosen on one rank either
    c2 = [0.0, 1.0, 1.0, 1.0, 1.0, 9.0]
    assert [k for k, _ in nat.plan_sweeps(8, 0, 8, 5, c2, ok)] == [4, 4] and nat.interval_depth(8, 5, c2, ok) == 4
    assert nat.hip_auto_depth("heat7", "f64", 2048, 2048, 2048, 5, 12) == 5
    assert nat.hip_auto_depth("heat7", "f64", 2048, 2048, 2048, 5, 12, nranks=8) == 4
    assert nat.hip_auto_depth("heat7", "f64", 2048, 2048, 2048, 5, 10, nranks=8) == 5
    assert nat.hip_auto_depth("heat7", "f32", 1024, 1024, 1024, 5, 0, nranks=8) == 5
    assert auto_temporal(m.heat3d(n=2048, dtype="f64"), 8, "hip", residual_every=12) == 4
    assert auto_temporal(m.heat3d(n=2048, dtype="f64"), 1, "hip", residual_every=12) == 5
    assert auto_temporal(m.heat3d(n=2048, dtype="f64"), 8, "hip", residual_every=10) == 5


def test_bench_pencil_candidates_fuse_at_most_four_steps():
    """bench.py gates and times (z, y) pencil candidates at their own depth: the slabs' fp32 depth 5
    has no pencil kernel (heat7_wxk's pencil copies fuse 3 / 4 steps), so a pencil candidate run at
    5 failed its gate (round-5 rehearsal, profiles/r05_session_y/)."""
    import importlib.util

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.depth_for_layout(5, 2, True) == 4 and bench.depth_for_layout(5, 1, True) == 5
    assert bench.depth_for_layout(3, 2, True) == 3 and bench.depth_for_layout(4, 4, True) == 4
    assert bench.depth_for_layout(5, 2, False) == 5  # (CPU pencils fuse any depth)


def test_warm_kernels_is_a_noop_on_cpu():
    import mpi_cuda_process_amd as m

    prob = m.heat3d(nx=24, ny=10, nz=12)
    with m.Simulation(prob, device="cpu", ranks=2) as sim:
        sim.init()
        before = sim.gather()
        sim.warm_kernels(7)
        assert np.array_equal(before, sim.gather())


# ---- (z, y) pencil decomposition on the CPU backend ------------------------------------------
@pytest.mark.parametrize("kind", ["heat7", "box27"])
@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("ranks,py", [(4, 2), (8, 2), (8, 4), (6, 3), (2, 2)])
@pytest.mark.parametrize("temporal", [1, 2, 3])
def test_pencil_bitwise_equals_single_rank(mdfx, kind, dtype, ranks, py, temporal):
    # pz x py pencils (2x2, 4x2, 2x4, 2x3, 1x2): two-phase exchange (y faces, then z faces with the
    # y ghost rows, which carries the edge / corner cells box27 reads) must reproduce P = 1 bitwise
    prob = (m.heat3d if kind == "heat7" else m.box27)(nx=20, ny=18, nz=16, dtype=dtype)
    with m.Simulation(prob, device="cpu") as sim:
        ref = sim.init().run(7).gather()
    with m.Simulation(prob, device="cpu", ranks=ranks, py=py, temporal=temporal) as sim:
        sim.init().run(7)
        assert sim.options["py"] == py
        assert np.array_equal(sim.gather(), ref)


def test_pencil_layouts_and_neighbours(mdfx):
    from mpi_cuda_process_amd.parallel.decomp import pencil_bounds, pencil_neighbors
    prob = m.heat3d(nx=12, ny=11, nz=9)
    with m.Simulation(prob, device="cpu", ranks=6, py=3, temporal=2) as sim:
        want = pencil_bounds(9, 11, 2, 3)
        for r in range(6):
            lay = sim.layout(r)
            (z0, z1), (y0, y1) = want[r]
            assert (lay["z0"], lay["z1"], lay["y0"], lay["y1"]) == (z0, z1, y0, y1)
            assert lay["hy"] == lay["halo"] == 2 and lay["nyl"] == y1 - y0
            assert lay["rows"] == lay["nyl"] + 2 * lay["hy"]
            assert lay["plane"] == lay["pitch"] * lay["rows"]
            assert sim.read_local(r).shape == (z1 - z0, y1 - y0, 12)
            assert tuple(sim.view(r).shape) == (lay["planes"], lay["rows"], lay["pitch"])
    assert pencil_neighbors(0, 2, 3) == (-1, 3, -1, 1)
    assert pencil_neighbors(4, 2, 3) == (1, -1, 3, 5)
    assert pencil_neighbors(5, 2, 3) == (2, -1, 4, -1)


def test_pencil_overlap_residual_and_sync_debug(mdfx):
    prob = m.box27(nx=18, ny=16, nz=14)
    outs, res = [], []
    for kw in (dict(overlap=True), dict(overlap=False), dict(sync_debug=True)):
        with m.Simulation(prob, device="cpu", ranks=4, py=2, residual_every=3, **kw) as sim:
            sim.init().run(6)
            outs.append(sim.gather())
            res.append(sim.residual)
    with m.Simulation(prob, device="cpu", residual_every=3) as sim:
        sim.init().run(6)
        want = sim.residual
    assert all(np.array_equal(outs[0], o) for o in outs[1:])
    assert all(abs(r - want) <= 1e-12 * max(1.0, want) for r in res)


def test_pencil_checkpoint_redecomposes(mdfx, tmp_path):
    # pencils -> slabs -> other pencils: every load gathers the row blocks it owns from any layout
    prob = m.heat3d(nx=14, ny=12, nz=10)
    with m.Simulation(prob, device="cpu") as sim:
        ref = sim.init().run(9).gather()
    with m.Simulation(prob, device="cpu", ranks=4, py=2) as sim:
        sim.init().run(3)
        sim.save_checkpoint(str(tmp_path / "a"))
    hdr = json.load(open(os.path.join(tmp_path, "a", "slab_3.json")))
    assert (hdr["y0"], hdr["y1"]) == (6, 12)
    with m.Simulation(prob, device="cpu", ranks=3) as sim:
        sim.load_checkpoint(str(tmp_path / "a"))
        sim.run(3)
        sim.save_checkpoint(str(tmp_path / "b"))
    with m.Simulation(prob, device="cpu", ranks=6, py=3, temporal=2) as sim:
        sim.load_checkpoint(str(tmp_path / "b"))
        sim.run(3)
        assert np.array_equal(sim.gather(), ref)


def test_pencil_bad_configs_rejected(mdfx):
    with pytest.raises(RuntimeError):
        m.Simulation(m.heat3d(n=8), device="cpu", ranks=6, py=4)  # py must divide the rank count
    with pytest.raises(RuntimeError):
        m.Simulation(m.heat3d(nx=8, ny=3, nz=8), device="cpu", ranks=4, py=4)  # too few rows
    with pytest.raises(RuntimeError):
        m.Simulation(m.mdf2d(h=16, w=16), device="cpu", ranks=2, py=2)  # 2D grids have one row

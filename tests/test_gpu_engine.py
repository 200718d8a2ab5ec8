"""Engine on the MI355X: decomposition invariance, overlap/race differential tests, hipGraph
replay, residual, checkpoint — tiers T3 and T5 of SURVEY §4.3.

P virtual slabs on ONE GPU through the loopback transport exercise the same engine code path as
RCCL (halo stream, events, double buffering); results must be bitwise equal to P = 1.
"""

import os
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import mpi_cuda_process_amd as m  # noqa: E402
from mpi_cuda_process_amd.ops import reference  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBS = [m.heat3d(nx=96, ny=40, nz=37), m.box27(nx=80, ny=24, nz=23), m.mdf2d(h=61, w=130),
         m.life2d(h=70, w=300), m.heat3d(nx=64, ny=30, nz=26, dtype="f64")]


def _ids(p):
    return p.describe().replace(" ", "_")


def _run(prob, steps, **kw):
    with m.Simulation(prob, device="hip", **kw) as sim:
        sim.init()
        sim.run(steps)
        sim.synchronize()
        return sim.gather(), sim.residual


@pytest.mark.parametrize("prob", PROBS, ids=_ids)
def test_decomposition_invariance_loopback(hip, prob):
    base, _ = _run(prob, 7, ranks=1)
    for p in (2, 3, 5):
        got, _ = _run(prob, 7, ranks=p)
        assert np.array_equal(base, got), "P=%d differs from P=1" % p


@pytest.mark.parametrize("prob", PROBS[:4], ids=_ids)
def test_overlap_vs_serialized(hip, prob):
    """Race screen: overlapped two-stream schedule == fully serialised (sync after every phase)."""
    a, _ = _run(prob, 9, ranks=4, overlap=True)
    b, _ = _run(prob, 9, ranks=4, overlap=False, sync_debug=True)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("prob", PROBS[:4], ids=_ids)
def test_graph_replay_equals_eager(hip, prob):
    a, _ = _run(prob, 10, ranks=1, graph=False)
    b, _ = _run(prob, 10, ranks=1, graph=True)
    assert np.array_equal(a, b)
    c, _ = _run(prob, 11, ranks=1, graph=True)  # odd count: graph pairs + one eager step
    assert np.array_equal(c, _run(prob, 11, ranks=1)[0])
    # several slabs in one process fall back to eager steps (see Solver::run)
    e, _ = _run(prob, 10, ranks=3, graph=True)
    assert np.array_equal(a, e)


@pytest.mark.parametrize("prob", PROBS + [m.heat3d(nx=1024, ny=20, nz=40)], ids=_ids)
def test_warm_kernels_leaves_state_unchanged(hip, prob):
    """warm_kernels(steps) launches each fused depth (and the residual copy) of a run into the
    scratch buffer: a run after it is bitwise the run without it, on 1 and 3 slabs."""
    for ranks in (1, 3):
        a, ra = _run(prob, 11, ranks=ranks, residual_every=5)
        with m.Simulation(prob, device="hip", ranks=ranks, residual_every=5) as sim:
            sim.init()
            sim.warm_kernels(11)
            sim.run(11)
            sim.synchronize()
            b, rb = sim.gather(), sim.residual
        # (the residual is summed with atomics in no fixed order: equal to rounding)
        assert np.array_equal(a, b) and abs(ra - rb) <= 1e-12 * abs(ra), ranks


@pytest.mark.parametrize("prob", [PROBS[0], m.heat3d(nx=256, ny=20, nz=40)], ids=_ids)
def test_prepared_graphs_replay_without_capture(hip, prob):
    """prepare_graphs() captures both parities up front; later runs (any warmup parity, across
    init()) only replay, and the result equals eager stepping bitwise."""
    t = 3 if prob.nx >= 256 else 1
    eager = {}
    for steps in (5, 20):
        with m.Simulation(prob, device="hip", temporal=t) as sim:
            sim.init()
            sim.run(steps)
            eager[steps] = sim.gather()
    with m.Simulation(prob, device="hip", graph=True, temporal=t) as sim:
        sim.init()
        assert sim.prepare_graphs() == 2
        caps = sim.graph_captures
        sim.run(5)  # the driver's warmup: leaves the buffer parity odd
        r0 = sim.graph_replays
        sim.run(20)
        assert sim.graph_captures == caps, "a capture happened inside the timed run"
        assert sim.graph_replays - r0 == 20 // (2 * t)
        sim.init()  # keeps the captured cycles
        sim.run(20)
        assert sim.graph_captures == caps
        assert np.array_equal(sim.gather(), eager[20])
        sim.init()
        sim.run(5)
        assert np.array_equal(sim.gather(), eager[5])


def test_graph_with_residual_interleave(hip):
    prob = m.heat3d(nx=64, ny=16, nz=18)
    with m.Simulation(prob, device="hip", graph=True, residual_every=4) as sim:
        sim.init()
        sim.run(9)
        g = sim.gather()
        r = sim.residual
    with m.Simulation(prob, device="hip", residual_every=4) as sim:
        sim.init()
        sim.run(9)
        assert np.array_equal(g, sim.gather()) and r == sim.residual


def test_matches_torch_reference_multi_step(hip):
    prob = m.heat3d(nx=72, ny=36, nz=30)
    with m.Simulation(prob, device="hip", ranks=3) as sim:
        sim.init()
        u0 = torch.from_numpy(sim.gather()).cuda().double()
        sim.run(6)
        sim.synchronize()
        got = torch.from_numpy(sim.gather()).cuda().double()
    ref = reference.run("heat7", u0, 6)
    assert (got - ref).abs().max().item() < 1e-5


def test_residual_and_convergence(hip):
    prob = m.mdf2d(h=48, w=64)
    with m.Simulation(prob, device="hip", ranks=2, residual_every=1) as sim:
        sim.init()
        sim.run(1)
        u1 = sim.gather()
        r1 = sim.residual
        sim.run(1)
        u2 = sim.gather()
        r2 = sim.residual
    want = float(np.sqrt(((u2.astype(np.float64) - u1) ** 2).sum()))
    assert abs(r2 - want) <= 1e-9 * max(want, 1.0)
    assert r1 > 0 and r2 > 0


def test_cpu_and_gpu_engines_agree_bitwise(hip):
    for prob in PROBS[:4]:
        g, _ = _run(prob, 5, ranks=2)
        with m.Simulation(prob, device="cpu", ranks=3) as sim:
            sim.init()
            sim.run(5)
            c = sim.gather()
        assert np.array_equal(g, c), prob.describe()


def test_checkpoint_resume_redecomposes(hip, tmp_path):
    prob = m.heat3d(nx=64, ny=20, nz=24)
    ref, _ = _run(prob, 8, ranks=1)
    with m.Simulation(prob, device="hip", ranks=4) as sim:
        sim.init()
        sim.run(5)
        sim.save_checkpoint(str(tmp_path / "ck"))
    with m.Simulation(prob, device="hip", ranks=3) as sim:
        sim.load_checkpoint(str(tmp_path / "ck"))
        assert sim.steps == 5
        sim.run(3)
        got = sim.gather()
    assert np.array_equal(ref, got)


def test_rccl_transport_single_rank(hip):
    """The native RCCL transport initialises and runs (world size 1 on a 1-GPU box)."""
    prob = m.heat3d(nx=64, ny=16, nz=16)
    a, _ = _run(prob, 4, ranks=1, transport="rccl")
    b, _ = _run(prob, 4, ranks=1)
    assert np.array_equal(a, b)


def test_zero_copy_view(hip):
    prob = m.heat3d(nx=64, ny=8, nz=6)
    with m.Simulation(prob, device="hip") as sim:
        sim.init()
        v = sim.view(0)
        assert v.is_cuda and v.dtype == torch.float32
        lay = sim.layout(0)
        assert tuple(v.shape) == (lay["planes"], lay["ny"], lay["pitch"])
        dense = torch.from_numpy(sim.gather()).cuda()
        assert torch.equal(v[1:-1, :, :64], dense)


def test_watchdog_timeout_option(hip):
    prob = m.heat3d(nx=64, ny=16, nz=16)
    with m.Simulation(prob, device="hip", ranks=2, timeout_s=60.0) as sim:
        sim.init()
        sim.run(3)
        sim.synchronize()


_SERIAL_WORKER = r"""
import sys; sys.path.insert(0, %(root)r)
import numpy as np, torch
import mpi_cuda_process_amd as m
out = {}
for name, prob, kw in [("heat7", m.heat3d(nx=300, ny=70, nz=64), dict(ranks=4, temporal=2)),
                       ("box27", m.box27(nx=200, ny=40, nz=33, dtype="f64"), dict(ranks=3)),
                       ("life", m.life2d(h=500, w=1500), dict(ranks=5, temporal=2))]:
    with m.Simulation(prob, device="hip", residual_every=5, **kw) as sim:
        sim.init()
        sim.run(11)
        sim.synchronize()
        out[name] = sim.gather()
np.savez(%(out)r, **out)
"""


def test_serialized_runtime_equals_overlapped(hip, tmp_path):
    """the HIP runtime's own serialisation (AMD_SERIALIZE_KERNEL / _COPY = 3: every kernel
    and copy waits for the previous one) must not change a single bit of the overlapped multi-slab
    result: a missing event dependency would show up as a difference here."""
    import subprocess
    import sys

    res = {}
    for tag, extra in (("overlap", {}), ("serial", {"AMD_SERIALIZE_KERNEL": "3", "AMD_SERIALIZE_COPY": "3"})):
        out = str(tmp_path / ("%s.npz" % tag))
        env = dict(os.environ, **extra)
        p = subprocess.run([sys.executable, "-c", _SERIAL_WORKER % dict(root=ROOT, out=out)], env=env,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
        assert p.returncode == 0, p.stderr.decode()[-3000:]
        res[tag] = np.load(out)
    for k in ("heat7", "box27", "life"):
        assert np.array_equal(res["overlap"][k], res["serial"][k]), k


@pytest.mark.parametrize("prob,steps", [(m.heat3d(nx=300, ny=20, nz=24), 9), (m.mdf2d(h=200, w=1100), 19),
                                        (m.life2d(h=150, w=2500), 13), (m.box27(nx=100, ny=30, nz=20), 6)])
def test_advance_on_gpu_equals_cpu(hip, prob, steps):
    """The functional API on a GPU tensor (auto fused depth) == the CPU oracle, bitwise."""
    with m.Simulation(prob, device="cpu") as sim:
        sim.init()
        g0 = torch.from_numpy(sim.gather().copy())
    gpu = m.advance(prob, g0.cuda(), steps)
    cpu = m.advance(prob, g0, steps, temporal=1)
    assert gpu.is_cuda and torch.equal(gpu.cpu(), cpu)


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_sweep_plan_by_cost_on_gpu(hip, dtype):
    """On the GPU the residual stretch is cut by the measured sweep costs: 10 steps at depth 4 on
    1024-cell rows run 4 + 3 + 3 (4 + 4 + 2 would spend a sweep on the slow two-step kernel), the
    residual by the last sweep; narrower rows keep 4 + 4 + 2. Bitwise equal to single steps."""
    prob = m.heat3d(nx=1024, ny=20, nz=40, dtype=dtype)
    with m.Simulation(prob, device="hip", ranks=2, temporal=4, residual_every=10) as sim:
        assert sim.sweep_plan(20) == [(4, False), (3, False), (3, True)] * 2
        sim.init()
        sim.run(23)
        got, gr = sim.gather(), sim.residual
    with m.Simulation(prob, device="hip", temporal=1, residual_every=10) as sim:
        sim.init()
        sim.run(23)
        assert np.array_equal(got, sim.gather()) and abs(gr - sim.residual) <= 1e-9 * max(1.0, gr)
    with m.Simulation(m.heat3d(nx=512, ny=20, nz=40, dtype=dtype), device="hip", temporal=4 if dtype == "f32" else 3,
                      residual_every=10) as sim:
        assert sim.sweep_plan(10) == ([(4, False), (4, False), (2, True)] if dtype == "f32" else
                                      [(3, False), (3, False), (3, False), (1, True)])


def test_auto_temporal_on_gpu(hip):
    from mpi_cuda_process_amd.engine import auto_temporal

    assert auto_temporal(m.heat3d(n=64), 1, "hip") == 2
    assert auto_temporal(m.mdf2d(h=4096, w=64), 4, "hip") == 8
    assert auto_temporal(m.mdf2d(h=40, w=64), 4, "hip") == 2  # 40 rows over 4 slabs: shallower sweeps
    assert auto_temporal(m.life2d(h=4096, w=64), 2, "hip") == 12
    assert auto_temporal(m.life2d(h=40, w=64), 2, "hip") == 3  # 40 rows over 2 slabs: 12 -> 6 -> 3
    prob = m.life2d(h=400, w=1000)
    ref, _ = _sim_gather(prob, 21, temporal=1)
    got, t = _sim_gather(prob, 21, temporal=0, ranks=3)
    assert t == 12 and np.array_equal(ref, got)


def _sim_gather(prob, steps, **kw):
    with m.Simulation(prob, device="hip", **kw) as sim:
        sim.init()
        sim.run(steps)
        return sim.gather(), sim.temporal


@pytest.mark.parametrize("ranks", [1, 3])
def test_mdf_ref_precision_gpu_equals_cpu(hip, ranks):
    """The reference-precision MDF update (fp32 sum, fp64 scale and add) is bitwise the same on the
    gfx950 wave kernel and the CPU oracle, decomposed or not."""
    import numpy as np

    import mpi_cuda_process_amd as m

    prob = m.mdf2d(h=300, w=777, ref_precision=True).with_init(kind="random", seed=5, lo=-10.0, hi=110.0)
    out = {}
    for dev in ("cpu", "hip"):
        with m.Simulation(prob, device=dev, ranks=ranks if dev == "hip" else 1, residual_every=9) as sim:
            assert sim.temporal == 1
            sim.init()
            sim.run(9)
            out[dev] = (sim.gather(), sim.residual)
    assert np.array_equal(out["cpu"][0], out["hip"][0])
    assert abs(out["cpu"][1] - out["hip"][1]) <= 1e-9 * out["cpu"][1]


# ---- (z, y) pencils, virtual ranks on one GPU (loopback transport) ----------------------------
@pytest.mark.parametrize("ranks,py", [(4, 2), (8, 2), (8, 4)])
@pytest.mark.parametrize("temporal", [1, 3, 4])
@pytest.mark.parametrize("graph", [False, True])
def test_pencil_loopback_bitwise_equals_single_rank(hip, ranks, py, temporal, graph):
    # 2x2 / 4x2 / 2x4 pencils: the y faces as 2-D copies, the z faces after the y pulls of the z
    # neighbour; the fused heat7_wxk sweep over the pencil's row range (K = 3, 4)
    prob = m.heat3d(nx=1024, ny=88, nz=72)
    with m.Simulation(prob, device="hip") as sim:
        ref = sim.init().run(9).gather()
    with m.Simulation(prob, device="hip", ranks=ranks, py=py, temporal=temporal, graph=graph) as sim:
        sim.init()
        sim.prepare_graphs()
        sim.run(9)
        assert np.array_equal(sim.gather(), ref)


@pytest.mark.parametrize("prob,temporal", [(m.box27(nx=130, ny=44, nz=36), 1),
                                           (m.box27(nx=130, ny=44, nz=36, dtype="f64"), 1),
                                           (m.heat3d(nx=200, ny=51, nz=40, dtype="f64"), 1),
                                           (m.heat3d(nx=200, ny=51, nz=40, dtype="f64"), 3),
                                           (m.heat3d(nx=200, ny=51, nz=40), 3)],
                         ids=["box27-f32", "box27-f64", "heat7-f64", "heat7-f64-k3", "heat7-f32-k3"])
def test_pencil_loopback_other_stencils(hip, prob, temporal):
    with m.Simulation(prob, device="hip", residual_every=3) as sim:
        ref = sim.init().run(7).gather()
        rres = sim.residual
    with m.Simulation(prob, device="hip", ranks=6, py=3, temporal=temporal, residual_every=3) as sim:
        sim.init().run(7)
        assert np.array_equal(sim.gather(), ref)
        assert abs(sim.residual - rres) <= 1e-9 * rres


@pytest.mark.parametrize("ranks,py", [(4, 2), (8, 4)])
def test_pencil_loopback_fp64_k4(hip, ranks, py):
    # fp64 K = 4 pencils: heat7_wxk's 2 + 1-row bands inside, 2 + 2-row 2-wave strips along the y
    # neighbours; residual sweeps included, replayed cycles in between
    prob = m.heat3d(nx=256, ny=72, nz=64, dtype="f64")
    with m.Simulation(prob, device="hip", residual_every=8) as sim:
        ref = sim.init().run(17).gather()
        rres = sim.residual
    with m.Simulation(prob, device="hip", ranks=ranks, py=py, temporal=4, graph=True, residual_every=8) as sim:
        sim.init()
        sim.prepare_graphs()
        sim.run(17)
        assert np.array_equal(sim.gather(), ref)
        assert abs(sim.residual - rres) <= 1e-9 * rres


def test_pencil_headline_shape_matches_slabs(hip):
    # the 1024^3 fp32 grid as 4 x 2 pencils (520-row pencils: the fused sweep's band / z-chunk
    # geometry at the N = 8 shape) against the slab split of the same ranks
    prob = m.heat3d(n=1024)
    outs = []
    for py in (1, 2):
        with m.Simulation(prob, device="hip", ranks=8, py=py, temporal=4) as sim:
            sim.init().run(8)
            outs.append(sim.gather())
    assert np.array_equal(outs[0], outs[1])

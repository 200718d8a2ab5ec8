"""Device-resident multi-process halo exchange on ONE GPU: 2-3 processes (one slab each) share
cuda:0 and pull their neighbours' faces through HIP IPC mappings, ordered by device-side counters
(csrc/comm/ipc_transport.cpp). No host staging: the faces move device-to-device on the copy
engines, exactly as across GPUs. Plus the watchdog escalation (a spinning device kernel or a dead
peer ends in a non-zero exit, not a hang) and bench.py's own multi-process launch + gate.

Reference parity: the rank-pair halo exchange of MDF_kernel.cu:166-172,180-183 / kernel.cu:214-216,
228-230, which in the reference deadlocks."""

import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r"""
import os, sys, json
sys.path.insert(0, %(root)r)
import numpy as np
import torch, torch.distributed as dist
import mpi_cuda_process_amd as m
from mpi_cuda_process_amd.parallel.dist import init_distributed
env = init_distributed("gloo")
torch.cuda.set_device(0)
prob = %(prob)s
with m.Simulation(prob, device="hip", distributed=True, transport=%(transport)r, residual_every=%(resid)d,
                  temporal=%(temporal)d, devices=[0], graph=%(graph)s, timeout_s=60.0, py=%(py)d,
                  share_gpu=True) as sim:
    assert sim.transport == %(transport)r, sim.transport
    sim.init()
    sim.run(%(steps)d)
    sim.synchronize()
    g = sim.gather()
    st = torch.tensor([sim.folded_sweeps, sim.graph_captures, *sim.graph_wait_nodes], dtype=torch.int64)
    dist.all_reduce(st, op=dist.ReduceOp.MAX)  # (rank 0 has no lower neighbour and never folds)
    if env.rank == 0:
        np.save(%(out)r, g)
        json.dump({"residual": sim.residual, "nranks": sim.nranks, "folded": int(st[0]), "captures": int(st[1]),
                   "waits": [int(st[2]), int(st[3])]}, open(%(out)r + ".json", "w"))
dist.barrier()
dist.destroy_process_group()
"""


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(world, argv_of, env_extra=None, timeout=180, expect_ok=True):
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        env.update(env_extra or {})
        procs.append(subprocess.Popen(argv_of(r), env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      cwd=ROOT))
    outs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=timeout)
            outs.append(o.decode())
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    if expect_ok:
        for p, o in zip(procs, outs):
            assert p.returncode == 0, o
    return procs, outs


def _resid(graph, steps):
    # graph runs of 13 steps take a residual every 12, so their first sweeps form a non-residual
    # stretch that is captured and replayed (every 4 would make every K = 4 sweep a residual sweep,
    # which always runs eagerly); the last residual is step 12's either way, as in _reference
    return 12 if graph and steps >= 13 else 4


def _reference(prob, steps, temporal=1):
    import mpi_cuda_process_amd as m

    with m.Simulation(prob, device="hip", residual_every=4, temporal=temporal) as sim:
        sim.init()
        sim.run(steps)
        return sim.gather(), sim.residual


@pytest.mark.parametrize("world,temporal,graph", [(2, 1, False), (3, 1, False), (2, 2, False), (3, 2, False),
                                                  (3, 2, True), (2, 3, False), (3, 3, True),
                                                  (3, 4, False), (4, 4, True), (4, 3, False)])
def test_ipc_multiprocess_matches_single(hip, tmp_path, world, temporal, graph):
    import mpi_cuda_process_amd as m

    prob_src = "m.heat3d(nx=256, ny=40, nz=47)"
    out = str(tmp_path / "g.npy")
    steps = 13
    code = WORKER % dict(py=1, root=ROOT, prob=prob_src, out=out, temporal=temporal, graph=graph, steps=steps,
                         resid=_resid(graph, steps), transport="ipc")
    _spawn(world, lambda r: [sys.executable, "-c", code])
    got = np.load(out)
    ref, rres = _reference(eval(prob_src), steps)
    assert np.array_equal(got, ref)
    meta = json.load(open(out + ".json"))
    assert meta["nranks"] == world and abs(meta["residual"] - rres) <= 1e-9 * rres
    assert (meta["captures"] > 0) == graph, meta  # graph runs really replay


@pytest.mark.parametrize("transport,direct,world,temporal,graph", [
    ("ipc", "0", 3, 2, True), ("ipc", "0", 4, 4, False),          # mailbox protocol (blit copies)
    ("ipc_sdma", "1", 3, 2, True), ("ipc_sdma", "1", 4, 4, False),  # direct pulls on the SDMA engines
    ("ipc_sdma", "0", 3, 3, True)])                                # mailbox on the SDMA engines
def test_ipc_protocols_and_copy_engines(hip, tmp_path, transport, direct, world, temporal, graph):
    """Both ipc protocols (direct pulls from the neighbours' exported field buffers / mailboxes) on
    both copy engines (blit kernels / SDMA), the two pulls of a middle rank on two streams:
    bitwise equal to one process, residual included, eager and replayed."""
    prob_src = "m.heat3d(nx=256, ny=40, nz=47)"
    out = str(tmp_path / "g.npy")
    steps = 13
    code = WORKER % dict(py=1, root=ROOT, prob=prob_src, out=out, temporal=temporal, graph=graph, steps=steps,
                         resid=_resid(graph, steps), transport=transport)
    _spawn(world, lambda r: [sys.executable, "-c", code], env_extra={"MDFX_IPC_DIRECT": direct})
    import mpi_cuda_process_amd as m  # noqa: F401 (eval below)

    ref, rres = _reference(eval(prob_src), steps)
    assert np.array_equal(np.load(out), ref)
    meta = json.load(open(out + ".json"))
    assert abs(meta["residual"] - rres) <= 1e-9 * rres
    assert (meta["captures"] > 0) == graph, meta


@pytest.mark.parametrize("graph", [False, True])
def test_ipc_fp64_fused_k4_folded(hip, tmp_path, graph):
    """fp64 K = 4 sweeps (heat7_wxk 2 + 1-row bands, the lower boundary folded into the interior
    sweep) over three processes: bitwise equal to one process, residual included. Eager runs fold;
    captured cycles hold device spin-waits (the ipc exchange's) but none on a fold counter."""
    import mpi_cuda_process_amd as m

    prob_src = "m.heat3d(nx=256, ny=40, nz=50, dtype='f64')"
    out = str(tmp_path / "g.npy")
    steps = 13
    code = WORKER % dict(py=1, root=ROOT, prob=prob_src, out=out, temporal=4, graph=graph, steps=steps,
                         resid=_resid(graph, steps), transport="ipc")
    _spawn(3, lambda r: [sys.executable, "-c", code])
    ref, rres = _reference(eval(prob_src), steps)
    assert np.array_equal(np.load(out), ref)
    meta = json.load(open(out + ".json"))
    assert abs(meta["residual"] - rres) <= 1e-9 * rres
    if graph:
        assert meta["captures"] > 0 and meta["waits"][0] > 0 and meta["waits"][1] == 0, meta
    else:
        assert meta["folded"] > 0 and meta["captures"] == 0, meta


@pytest.mark.parametrize("transport,direct,graph", [("ipc", "", False), ("ipc", "", True),
                                                     ("ipc_sdma", "1", False), ("ipc_sdma", "0", False)])
def test_ipc_fp32_fused_k5_folded(hip, tmp_path, transport, direct, graph):
    """fp32 K = 5 sweeps (the default depth of the 3D 7-point: heat7_wxk in rows of 2 cells per lane,
    the lower boundary folded into the interior sweep) over three processes: bitwise equal to one
    process, residual included; eager runs fold, captured cycles never wait on a fold counter.
    ipc_sdma: the folded face read by the SDMA engines, which bypass the L2 like a remote GPU's
    pull over xGMI (direct pulls from the field buffers, and the mailbox protocol's local publish
    copy): the face must have been written back by the time the halo stream's counter wait ends."""
    import mpi_cuda_process_amd as m

    prob_src = "m.heat3d(nx=300, ny=45, nz=66)"
    out = str(tmp_path / "g.npy")
    steps = 20  # (residual every 10 / 20: K = 5 sweeps throughout, the last residual step 20's as in _reference)
    code = WORKER % dict(py=1, root=ROOT, prob=prob_src, out=out, temporal=5, graph=graph, steps=steps,
                         resid=20 if graph else 10, transport=transport)
    _spawn(3, lambda r: [sys.executable, "-c", code], env_extra={"MDFX_IPC_DIRECT": direct} if direct else None)
    ref, rres = _reference(eval(prob_src), steps)
    assert np.array_equal(np.load(out), ref)
    meta = json.load(open(out + ".json"))
    assert abs(meta["residual"] - rres) <= 1e-9 * rres
    if graph:
        assert meta["captures"] > 0 and meta["waits"][0] > 0 and meta["waits"][1] == 0, meta
    else:
        assert meta["folded"] > 0 and meta["captures"] == 0, meta


@pytest.mark.parametrize("world,py,temporal,graph,transport,prob_src", [
    (4, 2, 4, False, "ipc", "m.heat3d(nx=256, ny=70, nz=47)"),   # 2 x 2 pencils, the fused K = 4 sweep
    (4, 2, 3, True, "ipc", "m.heat3d(nx=256, ny=70, nz=47)"),    # ... K = 3, replayed
    (4, 4, 4, True, "ipc", "m.heat3d(nx=256, ny=70, nz=47)"),    # 1 x 4 (y neighbours only)
    (6, 2, 3, False, "ipc_sdma", "m.heat3d(nx=130, ny=41, nz=44)"),  # 3 x 2, 2-D pulls on the SDMA engines
    (4, 2, 1, False, "ipc", "m.box27(nx=130, ny=41, nz=40, dtype='f64')"),  # edge / corner ghosts
])
def test_ipc_pencils_match_single(hip, tmp_path, world, py, temporal, graph, transport, prob_src):
    """(z, y) pencils, one process each, sharing the GPU: the y faces pulled as 2-D copies out of
    the neighbours' field buffers, then the z faces (carrying the fresh y ghost rows) once the z
    neighbours signal readyZ. Bitwise equal to one process, residual included."""
    import mpi_cuda_process_amd as m

    out = str(tmp_path / "g.npy")
    steps = 11
    code = WORKER % dict(py=py, root=ROOT, prob=prob_src, out=out, temporal=temporal, graph=graph, steps=steps,
                         resid=_resid(graph, steps), transport=transport)
    _spawn(world, lambda r: [sys.executable, "-c", code], env_extra={"MDFX_IPC_DIRECT": "1"})
    ref, rres = _reference(eval(prob_src), steps)
    assert np.array_equal(np.load(out), ref)
    meta = json.load(open(out + ".json"))
    assert abs(meta["residual"] - rres) <= 1e-9 * rres


@pytest.mark.parametrize("prob_src", ["m.mdf2d(h=203, w=300)", "m.life2d(h=150, w=257)",
                                      "m.box27(nx=130, ny=33, nz=40, dtype='f64')"])
def test_ipc_other_stencils(hip, tmp_path, prob_src):
    import mpi_cuda_process_amd as m

    out = str(tmp_path / "g.npy")
    code = WORKER % dict(py=1, root=ROOT, prob=prob_src, out=out, temporal=2, graph=False, steps=9, resid=4, transport="ipc")
    _spawn(3, lambda r: [sys.executable, "-c", code])
    ref, _ = _reference(eval(prob_src), 9)
    assert np.array_equal(np.load(out), ref)


def test_bench_self_launch_ipc_one_gpu(hip):
    """bench.py --gpus 2 with no launcher on a 1-GPU box: refused unless --share-gpu; with it, two
    ranks share cuda:0 over the ipc transport, pass the bitwise gate and report n_gpus = 2."""
    base = [sys.executable, os.path.join(ROOT, "bench.py"), "--n", "256", "--steps", "4", "--warmup", "2"]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    import torch

    if torch.cuda.device_count() == 1:
        t0 = time.time()
        p = subprocess.run(base + ["--gpus", "2"], env=env, capture_output=True, timeout=120, cwd=ROOT)
        assert p.returncode != 0 and time.time() - t0 < 60 and b"GPU" in p.stderr
    p = subprocess.run(base + ["--gpus", "2", "--share-gpu", "--transport", "ipc"], env=env, capture_output=True,
                       timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    lines = [l for l in p.stdout.decode().splitlines() if l.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["transport"] == "ipc" and rec["config"]["gate"]["passed"]
    assert rec["config"]["distinct_devices"] == 1


def test_watchdog_turns_a_spinning_kernel_into_an_exit(hip):
    """MDFX_FAULT=spin: a device kernel stops making progress (it would spin for 60 s). With a 5 s
    watchdog the process reports it and exits non-zero well before the kernel's own bound."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import mpi_cuda_process_amd as m\n"
            "sim = m.Simulation(m.heat3d(n=64), device='hip', timeout_s=5.0)\n"
            "sim.init(); sim.run(8); sim.synchronize()\n" % ROOT)
    t0 = time.time()
    p = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, MDFX_FAULT="spin@0:3"),
                       capture_output=True, timeout=120)
    el = time.time() - t0
    err = p.stderr.decode()
    assert p.returncode != 0 and "watchdog" in err, err[-2000:]
    assert el < 40, el


def test_ipc_dead_peer_is_an_error_not_a_hang(hip, tmp_path):
    """Rank 1 dies mid-run: rank 0's device wait times out, raises the error word, and the engine
    reports a transport failure and exits non-zero instead of hanging."""
    out = str(tmp_path / "g.npy")
    code = WORKER.replace("timeout_s=60.0", "timeout_s=5.0") % dict(
        py=1, root=ROOT, prob="m.heat3d(nx=128, ny=32, nz=40)", out=out, temporal=1, graph=False, steps=40, resid=4,
        transport="ipc")
    t0 = time.time()
    procs, outs = _spawn(2, lambda r: [sys.executable, "-c", code], env_extra={"MDFX_FAULT": "exit@1:3"},
                         timeout=150, expect_ok=False)
    assert procs[1].returncode == 42
    assert procs[0].returncode != 0, outs[0]
    assert time.time() - t0 < 120


def test_ipc_slabs_larger_than_2gib(hip):
    """1024^3 fp32 over 2 processes: each slab's field buffers are 2 GiB + 16 MiB. Mapping such a
    buffer through HIP IPC stalls forever under the HIP runtime PyTorch bundles (scripts/
    ipc_probe.py), so the transport exports only small face mailboxes: this run must finish."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-gpu", "--transport",
                        "ipc", "--n", "1024", "--steps", "4", "--warmup", "2", "--timeout", "30"],
                       env=env, capture_output=True, timeout=170, cwd=ROOT)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    rec = json.loads([l for l in p.stdout.decode().splitlines() if l.startswith("{")][0])
    assert rec["n_gpus"] == 2 and rec["config"]["gate"]["passed"] and rec["config"]["transport"] == "ipc"
    assert rec["config"]["ipc_protocol"] == "mailbox"


def test_ipc_direct_protocol_at_the_headline_size(hip):
    """1024^3 fp32 over 4 processes: field buffers of 1.1 GB map through HIP IPC, so the ranks pull
    each other's faces straight out of them (the direct protocol of the N >= 4 runs)."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--share-gpu", "--transport",
                        "ipc", "--n", "1024", "--steps", "8", "--warmup", "4", "--timeout", "30"],
                       env=env, capture_output=True, timeout=170, cwd=ROOT)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    rec = json.loads([l for l in p.stdout.decode().splitlines() if l.startswith("{")][0])
    cfg = rec["config"]
    assert rec["n_gpus"] == 4 and cfg["gate"]["passed"] and cfg["transport"] == "ipc"
    # every candidate passed its gate: the z slabs at the slab depth (5) and the 2 x 2 pencils at
    # theirs (4: pencils fuse at most 4 steps)
    runs = cfg["gate"]["runs"]
    assert {r["py"] for r in runs} == {1, 2} and all(r["passed"] for r in runs), runs
    assert cfg["ipc_protocol"] == "direct" and cfg["face_copy"] == "blit"
    # the timed run itself was checked on all four ranks against a full-grid naive run
    assert cfg["verified"]["passed"] and cfg["verified"]["ranks"] == 4 and cfg["verified"]["max_abs_diff"] == 0.0


def test_ipc_export_retry_path_runs_and_logs(hip, tmp_path):
    """MDFX_IPC_EXPORT_FAIL=2: the first two IPC exports of every process fail with "invalid
    argument"; the transport logs a diagnosis of the pointer (attributes, allocation range, overlap
    with imports it closed), retries, and the run stays bitwise equal to one process."""
    import mpi_cuda_process_amd as m

    prob_src = "m.heat3d(nx=128, ny=32, nz=40)"
    out = str(tmp_path / "g.npy")
    code = WORKER % dict(py=1, root=ROOT, prob=prob_src, out=out, temporal=2, graph=False, steps=6, resid=4,
                         transport="ipc")
    _, outs = _spawn(2, lambda r: [sys.executable, "-c", code], env_extra={"MDFX_IPC_EXPORT_FAIL": "2"})
    for o in outs:
        assert "hipIpcGetMemHandle succeeded after 2 retries" in o, o[-2000:]
        assert "allocation [" in o and "import(s) this process closed earlier" in o, o[-2000:]
    ref, _ = _reference(eval(prob_src), 6)
    assert np.array_equal(np.load(out), ref)


def test_ipc_refuses_two_engine_processes_on_one_gpu(hip, tmp_path):
    """Without share_gpu, two ipc engine processes on one GPU are refused at setup with a message
    (their device spin waits assume one process per GPU), on both ranks, quickly."""
    out = str(tmp_path / "g.npy")
    code = WORKER.replace(",\n                  share_gpu=True)", ")") % dict(
        py=1, root=ROOT, prob="m.heat3d(nx=128, ny=32, nz=40)", out=out, temporal=1, graph=False, steps=4,
        resid=4, transport="ipc")
    assert "share_gpu" not in code
    t0 = time.time()
    procs, outs = _spawn(2, lambda r: [sys.executable, "-c", code], timeout=120, expect_ok=False)
    assert all(p.returncode != 0 for p in procs), outs
    assert all("two engine processes on one GPU" in o for o in outs), outs
    assert time.time() - t0 < 90


def test_ipc_engines_rebuilt_in_turn_by_eight_processes(hip):
    """bench.py's trial loop builds and closes ipc engines in turn (slabs / pencils, blit / SDMA).
    With 8 processes on one GPU the 4th engine's hipIpcGetMemHandle failed ("invalid argument")
    until the transport's teardown made every rank unmap its neighbours' exports before any rank
    freed its own buffers (profiles/r04_session_e/)."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "ipc_churn.py"), "--world", "8"],
                       capture_output=True, timeout=240, cwd=ROOT)
    out = p.stdout.decode()
    if p.returncode != 0:
        err = p.stderr.decode()
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", "ipc_churn_stderr.log"), "w") as f:
            f.write(err)
        key = [l for l in err.splitlines() if "CHURN" in l or "HIP" in l or "mdfx" in l.lower()]
        raise AssertionError(out + "\n".join(key[:40]) + "\n" + err[-1500:])
    assert "engine 7 ipc_sdma py=2 ok" in out

"""Multi-process path on the CPU: one process per slab over torch.distributed (gloo), halo
exchange through the torch p2p callback transport, max-over-ranks timing — the same engine code
the GPU bench drives with RCCL. World size 2 and 3, rendezvous on 127.0.0.1.
"""

import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r"""
import os, sys, json
sys.path.insert(0, %(root)r)
import numpy as np
import torch.distributed as dist
import mpi_cuda_process_amd as m
from mpi_cuda_process_amd.parallel.dist import init_distributed
env = init_distributed("gloo")
prob = %(prob)s
with m.Simulation(prob, device="cpu", distributed=True, transport="torch", residual_every=3%(kw)s) as sim:
    sim.init()
    sim.run(7)
    g = sim.gather()
    if env.rank == 0:
        np.save(%(out)r, g)
        json.dump({"residual": sim.residual, "transport": sim.transport, "nranks": sim.nranks},
                  open(%(out)r + ".json", "w"))
dist.barrier()
dist.destroy_process_group()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(world, prob_src, out, kw=""):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER % dict(root=ROOT, prob=prob_src, out=out, kw=kw)],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(o.decode())
        assert p.returncode == 0, "\n".join(outs)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("prob_src", ["m.heat3d(nx=18, ny=10, nz=11)", "m.mdf2d(h=20, w=24)",
                                      "m.life2d(h=19, w=30)"])
def test_gloo_multiprocess_matches_single(mdfx, tmp_path, world, prob_src):
    import mpi_cuda_process_amd as m

    out = str(tmp_path / "g.npy")
    _launch(world, prob_src, out)
    got = np.load(out)
    prob = eval(prob_src)
    with m.Simulation(prob, device="cpu", residual_every=3) as sim:
        sim.init()
        sim.run(7)
        ref = sim.gather()
        ref_res = sim.residual
    assert np.array_equal(got, ref)
    import json

    meta = json.load(open(out + ".json"))
    assert meta["transport"] == "torch" and meta["nranks"] == world
    assert abs(meta["residual"] - ref_res) < 1e-9 * max(1.0, ref_res)


@pytest.mark.parametrize("world,py,prob_src", [(4, 2, "m.box27(nx=14, ny=12, nz=10)"),
                                               (4, 4, "m.heat3d(nx=16, ny=13, nz=9)"),
                                               (2, 2, "m.heat3d(nx=10, ny=12, nz=7, dtype='f64')")])
def test_gloo_multiprocess_pencils_match_single(mdfx, tmp_path, world, py, prob_src):
    # one process per pencil: y faces as strided (height, width) byte views over gloo, then z faces
    import json

    import mpi_cuda_process_amd as m

    out = str(tmp_path / "g.npy")
    _launch(world, prob_src, out, kw=", py=%d, temporal=2" % py)
    prob = eval(prob_src)
    with m.Simulation(prob, device="cpu", residual_every=3) as sim:
        ref = sim.init().run(7).gather()
        ref_res = sim.residual
    assert np.array_equal(np.load(out), ref)
    meta = json.load(open(out + ".json"))
    assert abs(meta["residual"] - ref_res) < 1e-9 * max(1.0, ref_res)


def test_bench_multiprocess_cpu_json(mdfx, tmp_path):
    """bench.py under a 2-process launch on CPU prints ONE JSON line from rank 0."""
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu",
                                       "--gpus", "2", "--n", "24", "--steps", "2", "--warmup", "1"],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE))
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e.decode()
    lines = [l for l in outs[0][0].decode().splitlines() if l.startswith("{")]
    assert len(lines) == 1 and not [l for l in outs[1][0].decode().splitlines() if l.startswith("{")]
    import json

    rec = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in rec
    assert rec["steps"] == 2 and rec["value"] > 0 and rec["config"]["grid"] == [24, 24, 24]


def _bench(args, env_extra=None, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MDFX_FORCE_DIST")}
    env.update({"OMP_NUM_THREADS": "2", **(env_extra or {})})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       timeout=timeout)
    return p.returncode, p.stdout.decode(), p.stderr.decode()


def test_bench_self_launches_ranks_cpu(mdfx):
    """--gpus N with no launcher environment spawns N ranks itself (never a silent 1-rank run),
    gates the decomposed engine bitwise against a full-grid run, and reports n_gpus = N."""
    import json

    rc, out, err = _bench(["--device", "cpu", "--gpus", "3", "--n", "32", "--steps", "2", "--warmup", "1"])
    assert rc == 0, err
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 3 and rec["config"]["ranks"] == 3
    gate = rec["config"]["gate"]
    run = gate["runs"][0]
    assert gate["passed"] and run["transport"] == "torch" and run["grid"][2] % 3 == 0


def test_bench_self_launches_8_ranks_cpu(mdfx):
    """The driver's N = 8 path rehearsed on the CPU: 8 self-launched gloo ranks, every rank gated
    bitwise against a full-grid run through the same transport, one JSON line with n_gpus = 8 that
    names the transport, the gate records and the timed-vs-trial ratio (the reference
    only ever meant 2 ranks, MDF_kernel.cu:29,37,155,189)."""
    import json

    rc, out, err = _bench(["--device", "cpu", "--gpus", "8", "--n", "64", "--steps", "4", "--warmup", "1"],
                          env_extra={"OMP_NUM_THREADS": "1"}, timeout=600)
    assert rc == 0, err
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    rec = json.loads(lines[0])
    cfg = rec["config"]
    assert rec["n_gpus"] == 8 and cfg["ranks"] == 8 and cfg["transport"] == "torch"
    assert cfg["gate"]["passed"] and all(r["passed"] for r in cfg["gate"]["runs"])
    assert cfg["gate"]["runs"][0]["grid"][2] % 8 == 0
    assert "timed_vs_trial" in cfg and rec["steps"] == 4 and rec["value"] > 0
    # slabs (z8) and 4 x 2 pencils are both gated and timed; the faster one is reported
    assert sorted({r["py"] for r in cfg["gate"]["runs"]}) == [1, 2]
    assert sorted({t["py"] for t in cfg["trials"]}) == [1, 2]
    assert cfg["py"] in (1, 2) and cfg["parallelism"].startswith("slab-z8" if cfg["py"] == 1 else "pencil-z4y2")
    # the timed run itself (not only the gate) was checked on every rank against a full-grid run,
    # and timed three times (the median reported)
    ver = cfg["verified"]
    assert ver["passed"] and ver["ranks"] == 8 and ver["max_abs_diff"] == 0.0 and ver["steps"] == [1, 4, 4, 4]
    assert len(cfg["repeats_ms_per_step"]) == 3 and rec["ms_per_step"] == sorted(cfg["repeats_ms_per_step"])[1]
    assert cfg["schedule"] in cfg["parallelism"]
    # self-diagnosis of the N > 1 run: every rank's phase split per sweep and its
    # face pulls timed alone, the selection phase's passes, and the bench's wall time
    ph, ln = cfg["phases"], cfg["links"]
    assert [p["rank"] for p in ph] == list(range(8)) and [l["rank"] for l in ln] == list(range(8))
    for p in ph:
        assert "error" not in p, p
        assert p["sweeps"] > 0 and p["step_us"] > 0 and p["interior_us"] >= 0
        assert {"boundary_us", "exchange_us", "exposed_us"} <= set(p)
    for r, l in enumerate(ln):
        assert "error" not in l, l
        npeer = 1 if r in (0, 7) else 2
        if cfg["py"] == 1:
            assert len(l["peers"]) == npeer and all(abs(q - r) == 1 for q in l["peers"])
        assert l["exchange_us"] > 0 and l["GBps_per_face"] > 0 and all(b > 0 for b in l["face_bytes"])
    assert cfg["trial_passes"] in (1, 2) and rec["wall_s"] > 0


def test_bench_n1_times_three_repeats_and_reports_the_median(mdfx):
    """At N = 1 too the timed window is three back-to-back repetitions; the median is reported
    (one 8-ms shot is noisy), and no N > 1 diagnostics are attached."""
    import json
    import statistics

    rc, out, err = _bench(["--device", "cpu", "--n", "24", "--steps", "3", "--warmup", "1"])
    assert rc == 0, err
    rec = json.loads([l for l in out.splitlines() if l.startswith("{")][0])
    cfg = rec["config"]
    reps = cfg["repeats_ms_per_step"]
    assert len(reps) == 3 and rec["ms_per_step"] == round(statistics.median(reps), 4)
    assert cfg["verified"]["steps"] == [1, 3, 3, 3] and cfg["verified"]["passed"]
    assert cfg["phases"] is None and cfg["links"] is None and rec["wall_s"] > 0


def test_ipc_export_retry_loop_cpu(mdfx):
    """The ipc transport's export retry: "invalid argument" is retried and the count
    returned; one failure too many raises with the call named and the retries counted."""
    nat = mdfx.native()
    assert nat.ipc_export_retry_selftest(0) == 0
    assert nat.ipc_export_retry_selftest(3) == 3
    with pytest.raises(RuntimeError, match=r"hipIpcGetMemHandle.*after 2 retries"):
        nat.ipc_export_retry_selftest(5, max_retries=2)


def test_bench_json_reports_effective_graph_mode(mdfx):
    """--graph on where nothing can replay (CPU): the JSON's graph flag is false, the request is
    reported separately, and no capture or replay is counted in the timed region."""
    import json

    rc, out, err = _bench(["--device", "cpu", "--graph", "on", "--n", "24", "--steps", "4", "--warmup", "1"])
    assert rc == 0, err
    rec = json.loads([l for l in out.splitlines() if l.startswith("{")][0])
    cfg = rec["config"]
    assert cfg["graph"] is False and cfg["graph_requested"] is True
    assert cfg["graph_replays_timed"] == 0 and cfg["graph_captures_timed"] == 0


def test_bench_refuses_more_gpus_than_visible(mdfx):
    """No GPU here: asking for 2 HIP ranks fails fast instead of running on fewer devices."""
    rc, out, err = _bench(["--device", "hip", "--gpus", "2", "--n", "32", "--steps", "1"], timeout=120)
    assert rc != 0 and "GPU" in err and not [l for l in out.splitlines() if l.startswith("{")]


def test_bench_gate_catches_a_broken_rank(mdfx):
    """A NaN injected into rank 1 during the gate run makes the gate fail on every rank and the
    bench exit non-zero without printing a number."""
    rc, out, err = _bench(["--device", "cpu", "--gpus", "2", "--n", "32", "--steps", "2", "--warmup", "1"],
                          env_extra={"MDFX_FAULT": "nan@1:2"})
    assert rc != 0, out
    assert "gate FAILED" in err or "gate" in err
    assert not [l for l in out.splitlines() if l.startswith("{")]


def test_bench_verification_catches_a_fault_the_gate_missed(mdfx):
    """MDFX_FAULT=ghost@1:timed corrupts one ghost cell of rank 1 only after the timed run's warm-up:
    the gate passes, the verification of the timed run against the full-grid run fails on the ranks
    the fault reaches, and the bench exits non-zero without printing a number."""
    rc, out, err = _bench(["--device", "cpu", "--gpus", "2", "--n", "32", "--steps", "4", "--warmup", "1"],
                          env_extra={"MDFX_FAULT": "ghost@1:timed"})
    assert rc != 0, out
    assert "injected a ghost-plane fault" in err
    assert "verification FAILED" in err and "the gate passed" in err
    assert not [l for l in out.splitlines() if l.startswith("{")]


def test_rccl_gets_the_single_stream_schedule_and_folds_only_on_request(mdfx):
    """RCCL's grouped send / recv is stream work on the halo stream under every HIP runtime, so one
    slab per process gets the boundary-on-compute schedule with it, eager where the runtime cannot
    capture it (it used to fall back to the two-stream schedule under HIP 7.0). The
    folded lower boundary is NOT rccl's default (no run has shown RCCL's p2p kernels
    reading a face published by a mid-sweep counter); fold=1 (bench.py's gated `rccl_fold`
    candidate) asks for it, fold=0 refuses it for every transport."""
    nat = mdfx.native()
    tr = nat.rccl_traits()
    assert tr["stream_ordered"] is True
    assert tr["graph_capturable"] == (nat.hip_runtime_version() >= 70200000)
    assert tr["fold_by_default"] is False
    assert nat.fold_allowed(-1, tr["fold_by_default"]) is False
    assert nat.fold_allowed(1, tr["fold_by_default"]) is True
    assert nat.fold_allowed(-1, True) is True and nat.fold_allowed(0, True) is False
    assert nat.step_schedule(True, 1, tr["stream_ordered"], True) == "folded"
    assert nat.step_schedule(True, 1, tr["stream_ordered"], False) == "boundary-on-compute"
    # several slabs in one process, or a host-side exchange (torch / staged callbacks): two streams
    assert nat.step_schedule(True, 2, tr["stream_ordered"], False) == "two-stream"
    assert nat.step_schedule(True, 1, False, False) == "two-stream"
    assert nat.step_schedule(False, 1, True, True) == "serialised"


CONTROL = r"""
import os, sys, json, struct
sys.path.insert(0, %(root)r)
import torch.distributed as dist
from mpi_cuda_process_amd.parallel.dist import init_distributed, ControlPlane
env = init_distributed("gloo")
cp = ControlPlane()
# a control plane handed a non-gloo group (torchrun's default NCCL group) builds its own gloo group
_real = dist.get_backend
dist.get_backend = lambda g=None: "nccl" if g is None else _real(g)
cp2 = ControlPlane()
cp3 = ControlPlane()  # a second engine's control plane reuses the group (no new collective)
dist.get_backend = _real
own_gloo = cp2.group is not None and _real(cp2.group) == "gloo" and cp3.group is cp2.group
cb2 = cp2.callbacks()
s2 = cb2["allreduce_sum"](1.0)
cb = cp.callbacks()
# an IpcRecord-shaped byte string: magic, ints, embedded NULs, two 64-byte handles
rec = b"MDFXIPC2" + struct.pack("<iiiiQ", env.rank, 0, 1000 + env.rank, 0, 8 << 20) + bytes(64) + bytes([env.rank]) * 64
allr = cb["allgather"](rec)
ok = [len(x) == len(rec) and struct.unpack("<i", x[8:12])[0] == r and x[-1] == r for r, x in enumerate(allr)]
s = cb["allreduce_sum"](float(env.rank + 1))
mx = cb["allreduce_max"](float(env.rank))
cb["barrier"]()
json.dump({"ok": all(ok) and len(allr) == env.world and own_gloo and s2 == env.world, "sum": s, "max": mx},
          open(%(out)r + str(env.rank), "w"))
dist.destroy_process_group()
"""


def test_ipc_control_plane_marshalling_cpu(mdfx, tmp_path):
    """The ipc transport's host control plane (gloo): binary handle records with embedded NULs
    come back from allgather intact and in rank order; the residual all-reduces and the barrier
    work across 3 processes."""
    import json

    out = str(tmp_path / "cp")
    port = _free_port()
    procs = []
    for r in range(3):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="3", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([sys.executable, "-c", CONTROL % dict(root=ROOT, out=out)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    for p in procs:
        o, _ = p.communicate(timeout=120)
        assert p.returncode == 0, o.decode()
    for r in range(3):
        rec = json.load(open(out + str(r)))
        assert rec == {"ok": True, "sum": 6.0, "max": 2.0}


def test_ipc_peer_record_checks_cpu(mdfx):
    """The ipc transport's host-side checks of a neighbour's record, including the cross-device
    case (no GPU needed): same pid refused, face size mismatch refused, another device accepted only
    with peer access."""
    nat = mdfx.native()
    me = dict(rank=0, device=0, pid=100, face_bytes=4 << 20)
    ok = dict(rank=1, device=0, pid=101, face_bytes=4 << 20)
    assert nat.ipc_peer_problem(me, ok, 1, False) == ""
    assert "different processes" in nat.ipc_peer_problem(me, dict(ok, pid=100), 1, True)
    assert "face size" in nat.ipc_peer_problem(me, dict(ok, face_bytes=1 << 20), 1, True)
    assert "mismatch" in nat.ipc_peer_problem(me, dict(ok, rank=2), 1, True)
    assert "mismatch" in nat.ipc_peer_problem(me, dict(ok, magic_ok=False), 1, True)
    other = dict(ok, device=3)
    assert nat.ipc_peer_problem(me, other, 1, True) == ""
    why = nat.ipc_peer_problem(me, other, 1, False)
    assert "cannot access device 3" in why and "rccl" in why


def test_ipc_refuses_engine_processes_sharing_a_gpu_cpu(mdfx):
    """Two engine processes on one GPU are refused unless share_gpu (test-only): the ipc exchange's
    device spin waits need the hardware scheduler to run every producer queue.
    Every rank checks the same allgathered records, so all refuse together."""
    nat = mdfx.native()
    pci = ["0000:05:00.0", "0000:15:00.0", "0000:65:00.0", "0000:75:00.0"]
    node = [(1000 + r, pci[r]) for r in range(4)]  # one process per GPU: fine
    assert nat.ipc_shared_gpu_problem(node) == ""
    shared = node + [(1004, pci[1])]
    why = nat.ipc_shared_gpu_problem(shared)
    assert "ranks 1 and 4" in why and pci[1] in why and "share_gpu" in why
    assert nat.ipc_shared_gpu_problem(shared, True) == ""
    # no PCI id (an old runtime): nothing to compare, no refusal; one process on one GPU: fine
    assert nat.ipc_shared_gpu_problem([(1, ""), (2, "")]) == ""
    assert nat.ipc_shared_gpu_problem([(7, pci[0]), (7, pci[0])]) == ""


def test_ipc_transport_needs_hip(mdfx):
    import mpi_cuda_process_amd as m

    with pytest.raises(ValueError, match="ipc"):
        # distributed=True without a process group is refused before any native call
        m.Simulation(m.heat3d(n=8), device="cpu", distributed=True, transport="ipc")

"""The real multi-process engine path on ONE GPU: 2-3 processes (one slab each) share cuda:0 and
exchange halos through host-staged torch.distributed gloo p2p (RCCL refuses two ranks on one GPU).
Everything except the RCCL calls themselves is the code the 8-GPU bench runs: env bootstrap, slab
ownership, halo spans, halo-stream ordering, residual all-reduce, max-over-ranks timing. Plus the
distributed bench path with the native RCCL transport at world size 1 (MDFX_FORCE_DIST)."""

import json
import os
import socket
import subprocess
import sys

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
with m.Simulation(prob, device="hip", distributed=True, transport="staged", residual_every=4,
                  temporal=%(temporal)d, devices=[0]) as sim:
    sim.init()
    sim.run(9)
    sim.synchronize()
    g = sim.gather()
    if env.rank == 0:
        np.save(%(out)r, g)
        json.dump({"residual": sim.residual, "nranks": sim.nranks}, open(%(out)r + ".json", "w"))
dist.barrier()
dist.destroy_process_group()
"""


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(world, src, env_extra=None, timeout=300):
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        env.update(env_extra or {})
        procs.append(subprocess.Popen(src(r), env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, cwd=ROOT))
    outs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=timeout)
            outs.append(o.decode())
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o
    return outs


@pytest.mark.parametrize("world,temporal", [(2, 1), (3, 1), (2, 2), (3, 2), (3, 3)])
def test_multiprocess_gpu_matches_single(hip, tmp_path, world, temporal):
    import mpi_cuda_process_amd as m

    prob_src = "m.heat3d(nx=256, ny=40, nz=47)"
    out = str(tmp_path / "g.npy")
    code = WORKER % dict(root=ROOT, prob=prob_src, out=out, temporal=temporal)
    _spawn(world, lambda r: [sys.executable, "-c", code])
    got = np.load(out)
    with m.Simulation(eval(prob_src), device="hip", residual_every=4) as sim:
        sim.init()
        sim.run(9)
        ref = sim.gather()
        rres = sim.residual
    assert np.array_equal(got, ref)
    meta = json.load(open(out + ".json"))
    assert meta["nranks"] == world and abs(meta["residual"] - rres) <= 1e-9 * rres


def test_bench_distributed_rccl_world1(hip):
    """bench.py through the distributed path (gloo control plane + native RCCL transport; with
    --transport auto the short trials may pick ipc instead, so the transport is named)."""
    outs = _spawn(1, lambda r: [sys.executable, os.path.join(ROOT, "bench.py"), "--n", "256", "--steps", "6",
                                "--warmup", "2", "--transport", "rccl"], env_extra={"MDFX_FORCE_DIST": "1"})
    rec = json.loads([l for l in outs[0].splitlines() if l.startswith("{")][0])
    assert rec["value"] > 0 and "rccl" in rec["config"]["parallelism"]


def test_bench_staged_two_processes(hip):
    outs = _spawn(2, lambda r: [sys.executable, os.path.join(ROOT, "bench.py"), "--n", "256", "--steps", "4",
                                "--warmup", "2", "--gpus", "2", "--transport", "staged", "--share-gpu"],
                  env_extra={"HIP_VISIBLE_DEVICES": "0"})
    lines = [l for l in outs[0].splitlines() if l.startswith("{")]
    assert len(lines) == 1 and json.loads(lines[0])["n_gpus"] == 2


INITHANG = r"""
import os, sys, time
sys.path.insert(0, %(root)r)
import torch
import mpi_cuda_process_amd as m
from mpi_cuda_process_amd.parallel.dist import init_distributed
env = init_distributed("gloo", timeout_s=120)
torch.cuda.set_device(0)
t0 = time.time()
try:
    m.Simulation(m.heat3d(n=64), device="hip", distributed=True, transport="rccl", timeout_s=%(t)f, devices=[0])
except Exception as e:  # the bounded bootstrap gave up: report and exit non-zero
    print("BOOTSTRAP-FAILED after %%.1f s: %%s" %% (time.time() - t0, e), flush=True)
    os._exit(3)
print("BOOTSTRAP-OK", flush=True)
os._exit(0)
"""


def test_rccl_bootstrap_is_bounded(hip):
    """A rank that never joins the RCCL communicator (MDFX_FAULT=inithang@1: rank 1 stops right
    before ncclCommInitRankConfig) makes rank 0 abort its half-built communicator and exit non-zero
    within the watchdog bound instead of blocking in ncclCommInitRank forever."""
    import time

    t = 8.0
    port = _port()
    procs = []
    code = INITHANG % dict(root=ROOT, t=t)
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), MDFX_FAULT="inithang@1")
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, cwd=ROOT))
    try:
        t0 = time.time()
        o, _ = procs[0].communicate(timeout=t + 60)
        took = time.time() - t0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for p in procs:
            p.wait()
    out = o.decode()
    assert procs[0].returncode == 3, out
    assert "BOOTSTRAP-FAILED" in out and "never joined" in out, out
    assert took < t + 45, "rank 0 took %.1f s to give up" % took


@pytest.mark.timeout(360)
def test_bench_rccl_bootstrap_hang_exits_nonzero(hip):
    """bench.py --gpus 2 --transport auto with a rank that never joins RCCL: the gate marks rccl
    failed, and the run ends non-zero (no usable transport with a hung peer) instead of hanging."""
    import time

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["MDFX_FAULT"] = "inithang@1"
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-gpu", "--n", "128",
                        "--steps", "4", "--warmup", "2", "--timeout", "8"], env=env, capture_output=True, timeout=400,
                       cwd=ROOT)
    took = time.time() - t0
    assert p.returncode != 0, p.stdout.decode()
    assert not [l for l in p.stdout.decode().splitlines() if l.startswith("{")]
    assert took < 300, took


@pytest.mark.timeout(300)
def test_bench_auto_fallback_to_staged(hip):
    """--transport auto when every device transport fails its gate (MDFX_FAULT=gate:rccl,ipc,ipc_sdma):
    the host-staged transport is gated as a last resort and timed, and the JSON names it."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["MDFX_FAULT"] = "gate:rccl,ipc,ipc_sdma"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-gpu", "--n", "128",
                        "--steps", "4", "--warmup", "2", "--graph", "off"], env=env, capture_output=True, timeout=280,
                       cwd=ROOT)
    out = p.stdout.decode()
    assert p.returncode == 0, out + p.stderr.decode()
    rec = json.loads([l for l in out.splitlines() if l.startswith("{")][0])
    assert rec["config"]["transport"] == "torch" and rec["config"]["gate"]["passed"]
    runs = rec["config"]["gate"]["runs"]
    assert [r["transport"] for r in runs] == ["rccl", "ipc", "ipc_sdma", "staged"] and runs[-1]["passed"]

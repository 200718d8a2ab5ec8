"""The examples/ scripts run end to end (CPU here; the GPU tier runs them on the MI355X)."""

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples")


def _run(args, device, timeout=300):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    p = subprocess.run([sys.executable] + args + ["--device", device], stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, env=env, timeout=timeout, cwd=ROOT)
    assert p.returncode == 0, (p.stdout.decode()[-2000:], p.stderr.decode()[-2000:])
    return p.stdout.decode()


CASES = [
    ([os.path.join(EX, "life_glider.py"), "--h", "24", "--w", "40", "--generations", "16", "--ranks", "3"],
     "glider moved 4 cells diagonally: yes"),
    ([os.path.join(EX, "mdf_heat_2d.py"), "--h", "64", "--w", "64", "--tol", "1e-1", "--report", "200", "--ranks", "2"],
     "converged"),
    ([os.path.join(EX, "heat3d_distributed.py"), "--n", "32", "--steps", "20", "--report", "10"], "'metric': 'GCells/s'"),
]


@pytest.mark.parametrize("args,expect", CASES, ids=["life_glider", "mdf_heat_2d", "heat3d_distributed"])
def test_example_cpu(args, expect):
    assert expect in _run(args, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("args,expect", CASES, ids=["life_glider", "mdf_heat_2d", "heat3d_distributed"])
def test_example_gpu(hip, args, expect):
    assert expect in _run(args, "hip")


@pytest.mark.gpu
def test_example_distributed_ipc_two_ranks_one_gpu(hip):
    """heat3d_distributed.py under a 2-rank launch on one GPU with the ipc transport: the residual
    trace equals the single-process run's."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    args = [sys.executable, os.path.join(EX, "heat3d_distributed.py"), "--n", "96", "--steps", "20", "--report",
            "10", "--device", "hip"]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen(args + ["--transport", "ipc", "--share-gpu"], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, cwd=ROOT))
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e.decode()[-2000:]
    multi = [l for l in outs[0][0].decode().splitlines() if l.startswith("step")]
    single = [l for l in _run(args[1:-2], "hip").splitlines() if l.startswith("step")]
    assert multi == single and len(multi) == 2
    assert "'transport': 'ipc'" in outs[0][0].decode()

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

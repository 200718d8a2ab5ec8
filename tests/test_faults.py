"""Failure detection: injected faults must end a run with an error, never a hang.
The reference deadlocks forever in MPI_Send; here a dead or hung peer, or a
diverging solution, produces a clear error within seconds. Faults come from MDFX_FAULT
(csrc/engine/solver.cpp: exit | hang | nan @ rank : step)."""

import os
import shutil
import subprocess
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "bin", "mdfx")
MPIEXEC = shutil.which("mpiexec") or ("/opt/conda/bin/mpiexec" if os.path.exists("/opt/conda/bin/mpiexec") else None)


def _run(args, env, timeout=90):
    e = dict(os.environ, OMP_NUM_THREADS="2")
    e.update(env)
    t0 = time.time()
    p = subprocess.run(args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=e, timeout=timeout, cwd="/tmp")
    return p, time.time() - t0


def test_nan_injection_trips_residual_guard():
    p, _ = _run([BIN, "--backend", "cpu", "--stencil", "7", "--n", "24", "--steps", "8", "--residual-every", "2",
                 "--ranks", "3"], {"MDFX_FAULT": "nan@1:3"})
    assert p.returncode != 0
    assert b"non-finite residual" in p.stderr and b"injecting fault 'nan'" in p.stderr


@pytest.mark.skipif(MPIEXEC is None, reason="no mpiexec in this image")
def test_dead_peer_is_an_error_not_a_hang():
    p, dt = _run([MPIEXEC, "-np", "3", BIN, "--backend", "cpu", "--stencil", "7", "--n", "24", "--steps", "20"],
                 {"MDFX_FAULT": "exit@1:4", "MDFX_PORT": str(33000 + os.getpid() % 700)})
    assert p.returncode != 0 and dt < 60
    assert b"peer closed the connection" in p.stderr or b"peer gone" in p.stderr


def test_hung_peer_times_out():
    """Rank 1 stops responding: rank 0 must fail within the TCP timeout instead of waiting forever.
    (Tearing down the hung rank is the launcher's job: torchrun does; the test kills it.)"""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(2):
        env = dict(os.environ, PMI_RANK=str(r), PMI_SIZE="2", MDFX_PORT=str(port), MDFX_FAULT="hang@1:3",
                   MDFX_TCP_TIMEOUT_S="2", OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([BIN, "--backend", "cpu", "--stencil", "5", "--h", "40", "--w", "40",
                                       "--steps", "20"], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      cwd="/tmp"))
    try:
        t0 = time.time()
        _, err = procs[0].communicate(timeout=60)
        assert procs[0].returncode != 0 and time.time() - t0 < 60
        assert b"timed out" in err
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()


def test_python_engine_nan_guard():
    import mpi_cuda_process_amd as m

    os.environ["MDFX_FAULT"] = "nan@0:2"
    try:
        # the fault table is read once per process: run in a child to keep this process clean
        code = ("import sys; sys.path.insert(0, %r)\n"
                "import mpi_cuda_process_amd as m\n"
                "sim = m.Simulation(m.heat3d(n=16), device='cpu', residual_every=1)\n"
                "sim.init()\n"
                "sim.run(6)\n") % ROOT
        p = subprocess.run(["python3", "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    finally:
        del os.environ["MDFX_FAULT"]
    assert p.returncode != 0 and b"non-finite residual" in p.stderr
    assert m is not None

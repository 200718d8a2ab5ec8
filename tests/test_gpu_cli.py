"""The native CLIs on the MI355X: the reference dialogue and print_array output are identical to the
CPU oracle's, with the GPU defaults (tuned kernels, fused two-step sweeps, overlap)."""

import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "bin")


def _run(args, stdin=""):
    p = subprocess.run(args, input=stdin.encode(), stdout=subprocess.PIPE, stderr=subprocess.PIPE, cwd=ROOT,
                       timeout=300)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    return p.stdout.decode()


@pytest.mark.parametrize("prog,extra", [("life", ["--init", "compat"]), ("life", []), ("mdf", ["--edge", "1"])])
def test_dialogue_print_gpu_equals_cpu(hip, prog, extra):
    gpu = _run([os.path.join(BIN, prog), "--print", "--ranks", "3"] + extra, "25\n70\n90\n")
    cpu = _run([os.path.join(BIN, prog), "--print", "--backend", "cpu"] + extra, "25\n70\n90\n")
    assert gpu == cpu and gpu.startswith("Enter desired number of generations:\n")


def test_json_reports_fused_sweeps_on_gpu(hip):
    rec = json.loads(_run([os.path.join(BIN, "mdfx"), "--stencil", "7", "--n", "128", "--steps", "10", "--json"]))
    assert rec["temporal"] == 2 and rec["n_gpus"] == 1 and rec["value"] > 0
    rec1 = json.loads(_run([os.path.join(BIN, "mdfx"), "--stencil", "7", "--n", "128", "--steps", "10", "--json",
                            "--temporal", "1"]))
    assert rec1["temporal"] == 1


def _port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch2(args, stdin=""):
    """Two CLI processes sharing cuda:0 (RANK / WORLD_SIZE launch, TCP rendezvous on 127.0.0.1);
    rank 0 alone reads stdin and prints. Returns rank 0's stdout."""
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MDFX_PORT=str(port))
        procs.append(subprocess.Popen(args, env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, cwd=ROOT))
    outs = []
    try:
        for r, p in enumerate(procs):
            o, e = p.communicate(input=stdin.encode() if r == 0 else b"", timeout=180)
            outs.append((o.decode(), e.decode()))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    return outs[0][0]


def test_cli_ipc_two_processes_match_one(hip):
    """The native CLI with one process per slab over the ipc transport (device-resident faces
    through HIP IPC mailboxes): the printed Life board and the heat residual equal one process's."""
    life = os.path.join(BIN, "life")
    single = _run([life, "--print"], "12\n40\n50\n")
    multi = _launch2([life, "--print", "--transport", "ipc", "--share-gpu"], "12\n40\n50\n")
    assert multi == single
    args = [os.path.join(BIN, "mdfx"), "--stencil", "7", "--n", "96", "--steps", "9", "--json", "--residual-every", "9"]
    one = json.loads(_run(args))
    two = json.loads([l for l in _launch2(args + ["--transport", "ipc", "--share-gpu"]).splitlines() if l.startswith("{")][0])
    assert two["transport"] == "ipc" and two["ranks"] == 2
    assert abs(two["residual"] - one["residual"]) <= 1e-9 * one["residual"]

"""`python -m mpi_cuda_process_amd`: same output as the native CLI, single process and under torchrun
(gloo, 2 ranks on the CPU)."""

import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "bin")


def _run(args, timeout=180):
    env = dict(os.environ, OMP_NUM_THREADS="2", HIP_VISIBLE_DEVICES="")
    p = subprocess.run(args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, cwd=ROOT, timeout=timeout)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    return p.stdout.decode()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_python_cli_print_matches_native():
    py = _run([sys.executable, "-m", "mpi_cuda_process_amd", "--device", "cpu", "--stencil", "life", "--h", "30",
               "--w", "40", "--steps", "9", "--print"])
    nat = _run([os.path.join(BIN, "life"), "--backend", "cpu", "--init", "life", "--h", "30", "--w", "40",
                "--steps", "9", "--print", "--quiet"])
    assert py == nat and "0" in py


def test_python_cli_json_virtual_ranks():
    out = _run([sys.executable, "-m", "mpi_cuda_process_amd", "--device", "cpu", "--n", "24", "--steps", "4",
                "--ranks", "3", "--temporal", "2", "--residual-every", "2", "--json"])
    rec = json.loads(out.strip().splitlines()[-1])
    assert rec["stencil"] == "heat7" and rec["grid"] == [24, 24, 24] and rec["value"] > 0 and rec["residual"] > 0


def test_python_cli_under_torchrun_matches_single_process(tmp_path):
    args = ["--device", "cpu", "--stencil", "life", "--h", "26", "--w", "30", "--steps", "7", "--print"]
    single = _run([sys.executable, "-m", "mpi_cuda_process_amd"] + args)
    # each rank's stdout goes to its own file (gloo prints connection chatter from both ranks)
    logs = str(tmp_path / "logs")
    _run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
          "--master-addr", "127.0.0.1", "--master-port", str(_port()), "--log-dir", logs, "--redirects", "1",
          "-m", "mpi_cuda_process_amd"] + args)
    outs = {}
    for root, _, files in os.walk(logs):
        if "stdout.log" in files:
            outs[os.path.basename(root)] = open(os.path.join(root, "stdout.log")).read()
    assert set(outs) == {"0", "1"}
    board = "".join(l for l in outs["0"].splitlines(keepends=True)
                    if not l.startswith("[Gloo]") and "peer ranks" not in l)
    assert board == single and "0" in single
    assert "0" not in "".join(l for l in outs["1"].splitlines() if "Gloo" not in l and "peer" not in l)

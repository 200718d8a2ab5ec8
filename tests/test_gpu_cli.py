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

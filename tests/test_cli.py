"""Native CLI compatibility: the reference's stdin dialogue, print_array output,
`mpirun -np N` launches (MPICH hydra PMI env, TCP halo transport on CPUs), flags, JSON metrics,
checkpoint/resume.
"""

import json
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "bin")
PROMPTS = ("Enter desired number of generations:\n"
           "Enter desired height of universe:\n"
           "Enter desired width of universe:\n")
MPIEXEC = shutil.which("mpiexec") or ("/opt/conda/bin/mpiexec" if os.path.exists("/opt/conda/bin/mpiexec") else None)


def run(args, stdin="", env=None, timeout=120):
    e = dict(os.environ, OMP_NUM_THREADS="2", HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", ""))
    e.update(env or {})
    p = subprocess.run(args, input=stdin.encode(), stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=e,
                       timeout=timeout, cwd=ROOT)
    assert p.returncode == 0, p.stderr.decode()
    return p.stdout.decode()


@pytest.fixture(scope="module", autouse=True)
def binaries():
    for b in ("mdf", "life", "mdfx"):
        if not os.path.exists(os.path.join(BIN, b)):
            pytest.fail("native CLIs are not built (make -j8)")


def test_dialogue_prompts_exact():
    out = run([os.path.join(BIN, "mdf"), "--backend", "cpu"], "3\n6\n9\n")
    assert out == PROMPTS  # the reference prints nothing else (print_array commented out)


def test_life_print_array_format():
    out = run([os.path.join(BIN, "life"), "--backend", "cpu", "--print"], "0\n5\n7\n")
    body = out[len(PROMPTS):]
    # '\n' + h rows of w chars + '\n' each + final '\n'  (kernel.cu:115-129)
    assert body.startswith("\n") and body.endswith("\n\n")
    rows = body[1:-1].split("\n")[:-1]
    assert len(rows) == 5 and all(len(r) == 7 for r in rows)
    # generation 0 is the glibc rand() board: frame dead
    assert rows[0].strip() == "" and rows[-1].strip() == ""
    assert all(r[0] == " " and r[-1] == " " for r in rows)


def test_life_compat_board_matches_native_init(mdfx):
    out = run([os.path.join(BIN, "life"), "--backend", "cpu", "--print"], "0\n12\n20\n")
    rows = out[len(PROMPTS):][1:-1].split("\n")[:-1]
    got = np.array([[1 if c == "0" else 0 for c in r] for r in rows], np.uint8)
    want = mdfx.native().life_compat_init(12, 20, 0.15, 1)
    assert np.array_equal(got, want)


def test_mdf_dirichlet_edges_print():
    # print_array prints '0' only for cells == 1: MDF values are 100 / heat -> blank board,
    # exactly the reference's (ill-typed) print on a float grid.
    out = run([os.path.join(BIN, "mdf"), "--backend", "cpu", "--print"], "2\n4\n6\n")
    body = out[len(PROMPTS):]
    assert body == "\n" + ("      \n" * 4) + "\n"


def test_flag_mode_json_and_residual():
    out = run([os.path.join(BIN, "mdfx"), "--backend", "cpu", "--stencil", "27", "--n", "16", "--steps", "4",
               "--residual-every", "2", "--json"])
    rec = json.loads(out.strip().splitlines()[-1])
    assert rec["stencil"] == "box27" and rec["grid"] == [16, 16, 16] and rec["steps"] == 4
    assert rec["value"] > 0 and rec["residual"] > 0


def test_ranks_invariance_via_print():
    a = run([os.path.join(BIN, "life"), "--backend", "cpu", "--print", "--h", "30", "--w", "40", "--steps", "9",
             "--init", "compat", "--quiet"])
    b = run([os.path.join(BIN, "life"), "--backend", "cpu", "--print", "--h", "30", "--w", "40", "--steps", "9",
             "--init", "compat", "--ranks", "4", "--quiet"])
    assert "0" in a and a == b


def test_checkpoint_resume_cli(tmp_path):
    ck = str(tmp_path / "ck")
    full = run([os.path.join(BIN, "mdfx"), "--backend", "cpu", "--stencil", "5", "--h", "20", "--w", "24",
                "--steps", "10", "--print", "--quiet"])
    run([os.path.join(BIN, "mdfx"), "--backend", "cpu", "--stencil", "5", "--h", "20", "--w", "24", "--steps",
         "6", "--checkpoint-every", "6", "--checkpoint-dir", ck, "--quiet", "--ranks", "3"])
    assert os.path.exists(os.path.join(ck, "slab_2.json"))
    resumed = run([os.path.join(BIN, "mdfx"), "--backend", "cpu", "--stencil", "5", "--h", "20", "--w", "24",
                   "--steps", "4", "--resume", ck, "--print", "--quiet", "--ranks", "2"])
    assert full == resumed


def test_fold_option():
    """--fold auto|on|off sets SolverOptions::fold (the RCCL transport folds only with `on`); other
    values are refused; the option does not change results (CPU ranks never fold)."""
    base = [os.path.join(BIN, "mdfx"), "--backend", "cpu", "--stencil", "7", "--n", "12", "--steps", "3", "--print",
            "--quiet", "--ranks", "2"]
    assert run(base + ["--fold", "off"]) == run(base + ["--fold", "on"]) == run(base)
    p = subprocess.run(base + ["--fold", "maybe"], stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    assert p.returncode != 0 and b"--fold takes auto, on or off" in p.stderr


def test_bad_option_fails():
    p = subprocess.run([os.path.join(BIN, "mdfx"), "--bogus"], stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    assert p.returncode != 0 and b"unknown option" in p.stderr


@pytest.mark.skipif(MPIEXEC is None, reason="no mpiexec in this image")
@pytest.mark.parametrize("np_", [2, 3])
def test_mpirun_life_matches_single_process(np_):
    single = run([os.path.join(BIN, "life"), "--backend", "cpu", "--print"], "15\n24\n33\n")
    multi = run([MPIEXEC, "-np", str(np_), os.path.join(BIN, "life"), "--backend", "cpu", "--print"],
                "15\n24\n33\n", env={"MDFX_PORT": str(31000 + np_ * 7 + os.getpid() % 500)})
    assert multi == single


@pytest.mark.skipif(MPIEXEC is None, reason="no mpiexec in this image")
def test_mpirun_heat7_json():
    out = run([MPIEXEC, "-np", "2", os.path.join(BIN, "mdfx"), "--backend", "cpu", "--stencil", "7", "--n", "20",
               "--steps", "3", "--json", "--residual-every", "3"],
              env={"MDFX_PORT": str(32000 + os.getpid() % 500)})
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["ranks"] == 2 and rec["transport"] == "tcp"
    single = run([os.path.join(BIN, "mdfx"), "--backend", "cpu", "--stencil", "7", "--n", "20", "--steps", "3",
                  "--json", "--residual-every", "3"])
    assert abs(json.loads(single.strip())["residual"] - rec["residual"]) < 1e-9 * rec["residual"]


def _read_dump(d):
    from mpi_cuda_process_amd.utils import read_checkpoint

    return read_checkpoint(d)


def test_dump_dim_profile_json_matches_python_engine(tmp_path):
    import mpi_cuda_process_amd as mm

    d = str(tmp_path / "dump")
    out = run([os.path.join(BIN, "mdfx"), "--backend", "cpu", "--dim", "3", "--n", "20", "--steps", "5", "--ranks",
               "3", "--dump", d, "--json", "--profile", "--trace"])
    rec = json.loads(out.strip().splitlines()[-1])
    assert rec["stencil"] == "heat7" and "phase_ms" in rec and 0 <= rec["halo_fraction"] <= 1
    assert rec["gcells_per_gpu"] > 0
    got, metas = _read_dump(d)
    assert len(metas) == 3 and all(m["step"] == 5 for m in metas)  # the dump precedes the profile steps
    with mm.Simulation(mm.heat3d(n=20), device="cpu", ranks=2) as sim:
        sim.init()
        sim.run(5)
        ref = sim.gather()
    assert np.array_equal(got, ref.reshape(got.shape))


def test_dim_bc_coef_aliases():
    a = run([os.path.join(BIN, "mdfx"), "--backend", "cpu", "--dim", "2", "--h", "12", "--w", "14", "--steps", "3",
             "--bc", "7", "--coef", "0.2", "--json"])
    b = run([os.path.join(BIN, "mdfx"), "--backend", "cpu", "--stencil", "5", "--h", "12", "--w", "14", "--steps",
             "3", "--edge", "7", "--r", "0.2", "--json"])
    assert json.loads(a)["stencil"] == "jacobi5" == json.loads(b)["stencil"]
    pa = run([os.path.join(BIN, "mdfx"), "--backend", "cpu", "--dim", "2", "--h", "12", "--w", "14", "--steps", "3",
              "--bc", "1", "--coef", "0.2", "--print", "--quiet"])
    pb = run([os.path.join(BIN, "mdfx"), "--backend", "cpu", "--stencil", "5", "--h", "12", "--w", "14", "--steps",
              "3", "--edge", "1", "--r", "0.2", "--print", "--quiet"])
    assert pa == pb and "0" in pa  # edges of value 1 print as '0'
    p = subprocess.run([os.path.join(BIN, "mdfx"), "--backend", "cpu", "--dim", "2", "--stencil", "7"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    assert p.returncode != 0 and b"--dim" in p.stderr


def test_utils_format_array_and_checkpoint_reader(tmp_path):
    """utils.format_array reproduces the native print_array bytes; read_checkpoint reassembles any
    decomposition and rejects incomplete directories."""
    import mpi_cuda_process_amd as mm
    from mpi_cuda_process_amd.utils import format_array, read_checkpoint

    ck = str(tmp_path / "ck")
    out = run([os.path.join(BIN, "life"), "--backend", "cpu", "--init", "life", "--h", "30", "--w", "40", "--steps",
               "5", "--print", "--quiet", "--ranks", "3", "--dump", ck])
    grid, metas = read_checkpoint(ck)
    assert len(metas) == 3 and grid.shape == (30, 1, 40) and format_array(grid) == out
    with mm.Simulation(mm.life2d(h=30, w=40), device="cpu") as sim:
        sim.init()
        sim.run(5)
        assert np.array_equal(sim.gather(), grid)
    os.remove(os.path.join(ck, "slab_1.json"))
    with pytest.raises(ValueError):
        read_checkpoint(ck)


@pytest.mark.parametrize("stencil,temporal", [("7", "2"), ("27", "1")])
def test_pencils_via_dump_match_slabs(tmp_path, stencil, temporal):
    # --py 2 / --py 3 pencils (host transport) dump the same grid as one slab; the dump reader places
    # every pencil's (z, y) block
    from mpi_cuda_process_amd.utils.checkpoint import read_checkpoint

    base = [os.path.join(BIN, "mdfx"), "--backend", "cpu", "--stencil", stencil, "--nx", "18", "--ny", "16",
            "--nz", "14", "--steps", "5", "--temporal", temporal, "--quiet"]
    run(base + ["--dump", str(tmp_path / "a")])
    run(base + ["--ranks", "4", "--py", "2", "--dump", str(tmp_path / "b")])
    run(base + ["--ranks", "6", "--py", "3", "--dump", str(tmp_path / "c")])
    a, _ = read_checkpoint(str(tmp_path / "a"))
    b, mb = read_checkpoint(str(tmp_path / "b"))
    c, _ = read_checkpoint(str(tmp_path / "c"))
    assert sorted((m["y0"], m["y1"]) for m in mb)[0] == (0, 8)
    assert np.array_equal(a, b) and np.array_equal(a, c)

"""Native unit tests (csrc/tests/test_main.cpp) as built, and under host AddressSanitizer +
UndefinedBehaviorSanitizer (make asan; host code only — GPU sanitizers are not available on the
MI355X pool). CPU tier: the GPU is hidden so the sanitizer run never touches a device."""

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "bin")


def _run(name, extra_env=None):
    exe = os.path.join(BIN, name)
    if not os.path.exists(exe):
        pytest.fail("%s is not built (make -j8 all)" % name)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="", OMP_NUM_THREADS="4")
    env.update(extra_env or {})
    p = subprocess.run([exe], stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, timeout=600)
    assert p.returncode == 0, p.stderr.decode()[-4000:]
    return p.stdout.decode() + p.stderr.decode()


def test_native_unit_tests_cpu():
    assert "all passed" in _run("mdfx_tests")


def test_native_unit_tests_asan_ubsan():
    if not os.path.exists(os.path.join(BIN, "mdfx_tests_asan")):  # not part of the default build
        subprocess.run(["make", "-C", ROOT, "-j8", "asan"], check=True, timeout=1500,
                       stdout=subprocess.DEVNULL)
    out = _run("mdfx_tests_asan", {"ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1",
                                   "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})
    assert "all passed" in out and "runtime error" not in out


def test_cmake_configures(tmp_path):
    """CMakeLists.txt (the embeddable build) configures against /opt/rocm (hip, rccl, OpenMP);
    the full build is exercised by scripts/cmake_build.sh."""
    import shutil

    if shutil.which("cmake") is None:
        pytest.skip("cmake not installed")
    p = subprocess.run(["cmake", "-S", ROOT, "-B", str(tmp_path / "b"), "-G", "Ninja"], stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, timeout=300)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    assert (tmp_path / "b" / "build.ninja").exists()


@pytest.mark.gpu
def test_native_device_checks_on_gpu(hip):
    """The device-check build (make devcheck): every tuned-kernel load and store in the native GPU
    tests (all stencils, single and fused steps, x-tiled rows, P = 1..4, graphs) stays inside its
    allocation. Violations are counted on the device, not trapped, so this cannot fault the GPU."""
    exe = os.path.join(BIN, "mdfx_tests_devcheck")
    if not os.path.exists(exe):
        pytest.fail("mdfx_tests_devcheck is not built (make -j8 devcheck, on the CPU before the GPU run)")
    p = subprocess.run([exe], stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=900)
    out = p.stdout.decode() + p.stderr.decode()
    assert p.returncode == 0, out[-4000:]
    assert "all passed (cpu + gpu)" in out and "device checks: 0 out-of-allocation accesses" in out

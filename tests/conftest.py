import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) HIP device")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def mdfx():
    import mpi_cuda_process_amd as m

    m.native()
    return m


@pytest.fixture(scope="session")
def hip(mdfx):
    if not mdfx.hip_available():
        pytest.fail("GPU test selected but no HIP device is available")
    return mdfx


@pytest.fixture
def knob(monkeypatch):
    """Set an MDFX_* kernel knob for one test: the native layer caches the knobs, so the cache is
    re-read after every change and again (restored environment) after the test."""
    import mpi_cuda_process_amd as m

    def set_knob(name, value):
        monkeypatch.setenv(name, str(value))
        m.native().reload_knobs()

    yield set_knob
    monkeypatch.undo()
    m.native().reload_knobs()

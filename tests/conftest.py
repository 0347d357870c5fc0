import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "bwa-mem-harp2_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def built():
    """Make sure the native artefacts exist (build once per session)."""
    lib = os.path.join(PKG, "lib", "libsmemgpu.so")
    orc = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not (os.path.exists(lib) and os.path.exists(orc)):
        import __graft_entry__
        __graft_entry__.build()
    return True


@pytest.fixture(scope="session")
def gpu_device(built):
    import smemgpu
    if smemgpu.device_count() < 1:
        pytest.fail("no HIP device visible to a -m gpu test")
    return 0

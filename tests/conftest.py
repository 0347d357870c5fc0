import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "bwa-mem-harp2_amd")
for p in (PKG, ROOT, os.path.join(ROOT, "tests")):  # tests/: shared helpers between test modules
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def _lib_is_current(lib: str) -> bool:
    """The .so's compiled-in source hash equals the hash of the sources beside
    it (a stale library pushed with the tree is rebuilt, never tested)."""
    if not os.path.exists(lib):
        return False
    import subprocess
    # in a child process: a loaded .so cannot be replaced in this one
    code = ("import smemgpu,sys; h = smemgpu.source_hash(); "
            "sys.exit(0 if smemgpu.build_id() in (h, h + '-ab') else 1)")
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([PKG, ROOT]))
    return subprocess.run([sys.executable, "-c", code], env=env).returncode == 0


@pytest.fixture(scope="session")
def built():
    """Make sure the native artefacts exist and are built from the current
    sources (build once per session)."""
    # SMEMGPU_LIB may name the A/B build (make AB=1: lib_ab/, build id "<hash>-ab")
    lib = os.environ.get("SMEMGPU_LIB") or os.path.join(PKG, "lib", "libsmemgpu.so")
    orc = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not (_lib_is_current(lib) and os.path.exists(orc)):
        import __graft_entry__
        __graft_entry__.build()
    import smemgpu
    h = smemgpu.source_hash()
    assert smemgpu.build_id() in (h, h + "-ab"), "libsmemgpu.so is not the build of these sources"
    return True


@pytest.fixture(scope="session")
def gpu_device(built):
    import smemgpu
    if smemgpu.device_count() < 1:
        pytest.fail("no HIP device visible to a -m gpu test")
    return 0

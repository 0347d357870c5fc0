"""smem_launch_offsets (the size -> offset scan every compaction uses: seeding,
SA lookup, chaining, chain2aln) against numpy's cumsum, at sizes around the
tile (2048) and tile-of-tiles (2048^2) boundaries.  Device memory comes from
libamdhip64 directly (the runtime libsmemgpu itself uses)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip(gpu_device):
    import smemgpu
    smemgpu.lib.load()
    h = C.CDLL("libamdhip64.so")
    h.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    h.hipFree.argtypes = [C.c_void_p]
    h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    h.hipDeviceSynchronize.argtypes = []
    so = smemgpu.lib.load()
    so.smem_launch_offsets.restype = C.c_int
    so.smem_launch_offsets.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.POINTER(C.c_size_t), C.c_void_p]
    return h


def _dev(hip, nbytes):
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), max(nbytes, 8)) == 0
    return p


@pytest.mark.parametrize("n", [0, 1, 7, 2047, 2048, 2049, 100_000, 2048 * 2048 - 1, 2048 * 2048 + 5, 9_000_001])
def test_offsets_scan(hip, n):
    from smemgpu import lib
    so = lib.load()
    rng = np.random.default_rng(n)
    a = rng.integers(0, 1 << 40, size=n, dtype=np.uint64) if n % 2 else rng.integers(0, 300, size=n, dtype=np.uint64)
    tmp = C.c_size_t(0)
    assert so.smem_launch_offsets(None, None, n, None, C.byref(tmp), None) == 0
    d_in, d_out, d_tmp = _dev(hip, 8 * n), _dev(hip, 8 * (n + 1)), _dev(hip, tmp.value)
    try:
        if n:
            assert hip.hipMemcpy(d_in, a.ctypes.data, 8 * n, 1) == 0  # hipMemcpyHostToDevice
        guard = np.full(n + 1, 0xDEADBEEF, np.uint64)
        assert hip.hipMemcpy(d_out, guard.ctypes.data, 8 * (n + 1), 1) == 0
        assert so.smem_launch_offsets(d_in, d_out, n, d_tmp, C.byref(tmp), None) == 0
        assert hip.hipDeviceSynchronize() == 0
        got = np.empty(n + 1, np.uint64)
        assert hip.hipMemcpy(got.ctypes.data, d_out, 8 * (n + 1), 2) == 0  # hipMemcpyDeviceToHost
        want = np.zeros(n + 1, np.uint64)
        want[1:] = np.cumsum(a, dtype=np.uint64)
        np.testing.assert_array_equal(got, want)
    finally:
        for p in (d_in, d_out, d_tmp):
            hip.hipFree(p)


def test_offsets_scan_small_temp(hip):
    from smemgpu import lib
    so = lib.load()
    n = 10_000
    tmp = C.c_size_t(8)  # too small for 5 tiles
    d = _dev(hip, 8 * (n + 1))
    try:
        assert so.smem_launch_offsets(d, d, n, d, C.byref(tmp), None) != 0
    finally:
        hip.hipFree(d)

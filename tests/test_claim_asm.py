"""The seeding kernel's hand-issued claim atomic (smem_kernels.hip WP_ISSUE,
OPT bit 8) must not have its destination VGPR read before the iteration's
`s_waitcnt vmcnt(0)`: LLVM does not track the result of an inline-asm VMEM
instruction, so this is checked on the machine code of the library the tests
load (tools/check_claim_wait.py).  CPU only: it disassembles."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import check_claim_wait as ccw  # noqa: E402

LIB = os.path.join(ROOT, "bwa-mem-harp2_amd", "lib", "libsmemgpu.so")


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists(f"{ccw.LLVM}/llvm-objdump"),
                    reason="library or LLVM tools missing")
def test_default_kernel_claim_waits():
    n, bad = ccw.run(LIB)
    assert n == 1, "expected exactly one hand-issued claim atomic in the default seeding kernel"
    assert bad == []


def _i(a, mn, ops):
    return (a, mn, ops)


def test_checker_flags_an_early_read():
    base = 0x1000
    ok = [_i(base, "global_atomic_add", "v4, v[2:3], v1, off sc0"),
          _i(base + 8, "v_mov_b32", "v5, v6"),
          _i(base + 12, "s_cbranch_execz", f"2 <k+0x{20:x}>"),
          _i(base + 16, "s_waitcnt", "vmcnt(0)"),
          _i(base + 20, "s_waitcnt", "vmcnt(0) lgkmcnt(0)"),
          _i(base + 24, "v_readlane_b32", "s0, v4, s1")]
    assert ccw.check(ok, base) == (1, [])
    early = list(ok)
    early[1] = _i(base + 8, "v_mov_b32", "v7, v4")  # a copy before the wait
    n, bad = ccw.check(early, base)
    assert n == 1 and len(bad) == 1
    ranged = list(ok)
    ranged[1] = _i(base + 8, "global_store_dwordx2", "v[3:4], v[8:9], off")  # inside a register range
    assert len(ccw.check(ranged, base)[1]) == 1
    branch = list(ok)
    branch[3] = _i(base + 16, "s_waitcnt", "vmcnt(1)")  # not a full wait: the branch's other path
    branch[4] = _i(base + 20, "s_nop", "0")               # reaches the read
    assert len(ccw.check(branch, base)[1]) == 1

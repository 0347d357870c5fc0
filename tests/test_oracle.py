"""CPU tests: pin the oracle (C restatement) against the reference's own
outputs, and check the index builder and the C ABI library without a GPU."""
import os
import re

import numpy as np
import pytest

from oracle import oracle
from tests import golden_data


@pytest.fixture(scope="module")
def fx(built):
    return golden_data.load()


@pytest.fixture(scope="module")
def oidx(fx):
    return oracle.OracleIndex(words=fx.index.words, primary=fx.index.primary, L2=fx.index.L2)


def test_fixture_manifest(fx):
    assert fx.genome.size == fx.manifest["genome"]["n_bp"]
    assert fx.reads.n == 1500
    names = [c["name"] for c in fx.cases]
    assert names == ["default", "noexact", "k14s20", "reseed", "k30"]


@pytest.mark.parametrize("case_i", range(5))
def test_oracle_matches_reference_golden(fx, oidx, case_i):
    """C restatement == compiled reference smem_next2 stream, byte for byte."""
    case = fx.cases[case_i]
    reads = fx.reads.subset(np.arange(case["n_reads"]))
    got, per, st = oracle.seed(oidx, reads.codes, reads.offs, threads=2, **case["opt"])
    assert got == fx.stream(case)
    assert st["n_intv"] == case["n_intv"] and st["n_calls"] == case["n_calls"]


def test_oracle_threads_invariant(fx, oidx):
    reads = fx.reads.subset(np.arange(300))
    a, _, sa = oracle.seed(oidx, reads.codes, reads.offs, threads=1)
    b, _, sb = oracle.seed(oidx, reads.codes, reads.offs, threads=7)
    assert a == b and sa == sb


def test_occ4_brute_force(fx, oidx):
    """orc_occ4 against a direct count over the unpacked BWT string."""
    words = fx.index.words
    n = fx.index.seq_len
    prim = fx.index.primary
    # unpack the $-free BWT from the interleaved layout
    nb = (n + 127) // 128
    sym = np.empty(n, dtype=np.uint8)
    for b in range(nb):
        w = words[b * 16 + 8: b * 16 + 16].astype(np.uint64)
        s = ((w[:, None] >> (np.uint64(2) * (15 - np.arange(16, dtype=np.uint64)))) & np.uint64(3)).reshape(-1)
        m = min(128, n - b * 128)
        sym[b * 128: b * 128 + m] = s[:m]
    cum = np.zeros((n + 1, 4), dtype=np.int64)
    for c in range(4):
        cum[1:, c] = np.cumsum(sym == c)
    rng = np.random.default_rng(0)
    ks = np.concatenate([rng.integers(0, n + 1, 3000), [0, 1, prim - 1, prim, prim + 1, n - 1, n]])
    for k in ks:
        k = int(k)
        kk = k - (k >= prim)
        want = cum[kk + 1]
        assert oidx.occ4(k).tolist() == want.tolist(), k
    assert oidx.occ4(-1).tolist() == [0, 0, 0, 0]


def test_index_builder_matches_reference(fx, tmp_path):
    """smem_bwt_build == `bwa index -a is` of the same FASTA, byte for byte."""
    import smemgpu
    idx = smemgpu.Index.build(fx.genome)
    p = str(tmp_path / "mine.bwt")
    idx.write(p)
    with open(p, "rb") as fh:
        assert fh.read() == fx.bwt_bytes


@pytest.mark.parametrize("n_bp,seed", [(1, 1), (7, 2), (128, 3), (1000, 4), (4099, 5)])
def test_index_builder_small_vs_reference(n_bp, seed, tmp_path, built):
    """Tiny genomes (bucket-boundary sizes) against the reference indexer."""
    if not oracle.ref_available():
        pytest.skip("reference harness not built (no /root/reference on this machine)")
    import smemgpu
    from smemgpu import synth
    g = synth.make_genome(n_bp, seed=seed, n_chrom=1)
    fa = str(tmp_path / "g.fa")
    synth.write_fasta(fa, g)
    oracle.ref_index(fa, str(tmp_path / "g"))
    idx = smemgpu.Index.build(g.codes)
    p = str(tmp_path / "mine.bwt")
    idx.write(p)
    assert open(p, "rb").read() == open(str(tmp_path / "g.bwt"), "rb").read()


def test_bwt_roundtrip(fx, tmp_path):
    import smemgpu
    p = str(tmp_path / "a.bwt")
    with open(p, "wb") as fh:
        fh.write(fx.bwt_bytes)
    idx = smemgpu.Index.read(p)
    assert idx.primary == fx.index.primary
    assert idx.seq_len == 2 * fx.genome.size
    q = str(tmp_path / "b.bwt")
    idx.write(q)
    assert open(q, "rb").read() == fx.bwt_bytes


def test_abi_exports_every_declared_symbol(built):
    """libsmemgpu.so loads without a GPU and exports every function
    include/smem_gpu.h declares (no compute calls here)."""
    import ctypes
    import smemgpu
    from smemgpu.lib import EXPORTED
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "smem_gpu.h")).read()
    declared = set(re.findall(r"^\s*(?:const\s+)?(?:int|void|char)\s*\*?\s*(smem_\w+)\s*\(", hdr, re.M))
    assert declared, "no declarations parsed"
    assert declared == set(EXPORTED)
    lib = smemgpu.load()
    for name in declared:
        assert hasattr(lib, name), name
        assert ctypes.cast(getattr(lib, name), ctypes.c_void_p).value


def test_no_device_is_an_error_not_a_fallback(built):
    """Without a GPU the product path refuses instead of computing on the CPU."""
    import smemgpu
    if smemgpu.device_count() > 0:
        pytest.skip("a GPU is visible")
    from smemgpu import synth
    idx = smemgpu.Index.build(synth.make_genome(2000, seed=1).codes)
    with pytest.raises(smemgpu.SmemError, match="SMEM_E_DEVICE"):
        smemgpu.Gpu(idx, device=0)

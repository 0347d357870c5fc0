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


@pytest.mark.parametrize("case_i", range(5))
def test_oracle_sa_matches_reference_golden(fx, oidx, case_i, tmp_path):
    """Restated bwt_sa == the compiled reference's bwt_sa for every seed
    occurrence mem_insert_seed generates from the golden stream."""
    from smemgpu import synth
    case = fx.cases[case_i]
    p = str(tmp_path / "g1.sa")
    with open(p, "wb") as fh:
        fh.write(fx.sa_bytes)
    osa = oracle.OracleSA(path=p)
    counts, k = oracle.sa_queries(synth.read_smgo(fx.stream(case)), case["opt"]["min_seed_len"], case["max_occ"])
    pos = osa.lookup(oidx, k)
    want = synth.read_smsa(fx.sa_stream(case))
    assert [w.size for w in want] == counts.tolist()
    assert np.array_equal(np.concatenate(want) if want else np.zeros(0, np.uint64), pos)
    assert pos.size == case["n_occ"]
    osa.close()


def test_sa_builder_matches_reference(fx, tmp_path):
    """smem_bwt_build_sa's .sa == `bwa index`'s .sa (bwt_cal_sa, interval 32), byte for byte."""
    import smemgpu
    idx, sa = smemgpu.Index.build_sa(fx.genome, sa_intv=32)
    p = str(tmp_path / "mine.sa")
    sa.write(p)
    assert open(p, "rb").read() == fx.sa_bytes
    back = smemgpu.SA.read(p)
    assert np.array_equal(back.samples, sa.samples) and back.sa_intv == 32
    with open(str(tmp_path / "mine.bwt"), "wb"):
        pass
    idx.write(str(tmp_path / "mine.bwt"))
    assert open(str(tmp_path / "mine.bwt"), "rb").read() == fx.bwt_bytes


@pytest.mark.parametrize("n_bp,seed,intv", [(1, 1, 32), (100, 2, 1), (2000, 3, 8), (3000, 4, 32), (3000, 4, 128)])
def test_sa_lookup_brute_force(n_bp, seed, intv, built):
    """Restated bwt_sa == the full suffix array (computed in Python) for every row."""
    import smemgpu
    from smemgpu import synth
    g = synth.make_genome(n_bp, seed=seed, n_chrom=1).codes
    idx, sa = smemgpu.Index.build_sa(g, sa_intv=intv)
    n = idx.seq_len
    text = np.concatenate([g, (3 - g[::-1])]).astype(np.uint8)
    # full SA of text$ by sorting suffixes (small n only)
    # suffixes of text$: a proper prefix sorts first, so "$" (the empty suffix) is smallest
    order = sorted(range(n + 1), key=lambda i: bytes(text[i:].tolist()))
    oidx = oracle.OracleIndex(words=idx.words, primary=idx.primary, L2=idx.L2)
    osa = oracle.OracleSA(sa=sa.samples, sa_intv=intv, seq_len=n)
    rows = np.arange(n + 1, dtype=np.uint64) if n < 3000 else np.random.default_rng(seed).integers(0, n + 1, 3000).astype(np.uint64)
    got = osa.lookup(oidx, rows)
    want = np.array([order[int(r)] if int(r) > 0 else (2 ** 64 - 1 + 0) for r in rows], dtype=np.uint64)
    # row 0 is the $ suffix: sa[0] = -1 makes bwt_sa return (steps - 1) mod 2^64 there, as the reference does
    nz = rows != 0
    assert np.array_equal(got[nz], want[nz])
    osa.close()
    oidx.close()


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


CHAINS = golden_data.chain_fixtures()


@pytest.mark.parametrize("g,case,ch", CHAINS, ids=[c["file"].split(".")[0] for _, _, c in CHAINS])
def test_oracle_chains_match_reference_golden(g, case, ch):
    """mem_chain (+ mem_chain_flt) restated (oracle/chain_oracle.c) over the
    golden seed sequence == the compiled reference's chains, byte for byte."""
    from smemgpu import synth
    lists = synth.read_smgo(golden_data.smgo(g, case))
    pos = synth.read_smsa(golden_data.smsa(g, case))
    seeds, off = oracle.chain_seeds(lists, pos, case["opt"]["min_seed_len"], case["max_occ"])
    got = oracle.chain(seeds, off, golden_data.l_pac(g), w=ch["w"], max_chain_gap=ch["max_chain_gap"],
                       min_seed_len=case["opt"]["min_seed_len"], mask_level=ch["mask_level"],
                       drop_ratio=ch["drop_ratio"], filter=ch["filter"], threads=4)
    assert got == golden_data.smch(ch)


def test_g2_fixture_is_repeat_dense():
    """g2 exists to reach multi-level chain trees, long filter sorts and
    duplicate chain keys; keep it that way"""
    from smemgpu import synth
    g, case, ch = [x for x in CHAINS if x[0] == "g2" and x[2]["name"] == "tight" and x[2]["filter"] == 0][0]
    chains = synth.read_smch(golden_data.smch(ch))
    assert max(len(r) for r in chains) > 120          # three tree levels
    assert sum(len(r) - len({p for p, _ in r}) for r in chains) > 0


def test_oracle_g2_streams_match_reference(tmp_path):
    """the restated seeding loop and bwt_sa on the repeat-dense genome"""
    from smemgpu import synth
    p = golden_data.files("g2", str(tmp_path))
    oi = oracle.OracleIndex(p["bwt"])
    osa = oracle.OracleSA(p["sa"])
    reads = synth.read_smrd(p["smrd"])
    for case in golden_data.genome_cases("g2"):
        data, _, _ = oracle.seed(oi, reads.codes, reads.offs, threads=4, **case["opt"])
        assert data == golden_data.smgo("g2", case)
        lists = synth.read_smgo(data)
        _, k = oracle.sa_queries(lists, case["opt"]["min_seed_len"], case["max_occ"])
        exp = np.concatenate(synth.read_smsa(golden_data.smsa("g2", case)))
        assert np.array_equal(osa.lookup(oi, k), exp)
    osa.close()
    oi.close()


def test_ksw_oracle_matches_reference_golden():
    """The restated ksw_extend2 (oracle/ksw_oracle.c) == the compiled reference's
    own ksw_extend2 (software/ksw.c:379) on 5000 extension problems."""
    from smemgpu import synth
    from tests import golden_data
    b = synth.read_smkt(golden_data.gz("ksw.smkt.gz"))
    want = synth.read_smkr(golden_data.gz("ksw.smkr.gz"))
    assert b.tasks.size == want.size == 5000
    assert np.array_equal(oracle.ksw(b), want)


def test_ksw_oracle_matches_reference_live(tmp_path):
    """Fresh problems under other scoring (a=2 b=3, o_del 5 e_del 2, o_ins 4
    e_ins 1), checked against the reference binary when it is built."""
    from smemgpu import synth
    if not oracle.ref_available():
        pytest.skip("oracle/_ref not built")
    g = synth.make_genome(100_000, seed=131, n_chrom=1)
    b = synth.make_ksw_tasks(g.codes, 1500, seed=132)
    b.mat = synth.bwa_scmat(2, 3)
    b.o_del, b.e_del, b.o_ins, b.e_ins = 5, 2, 4, 1
    p = str(tmp_path / "t.smkt")
    synth.write_smkt(p, b)
    oracle.ref_ksw(p, str(tmp_path / "r.smkr"))
    want = synth.read_smkr(open(tmp_path / "r.smkr", "rb").read())
    assert np.array_equal(oracle.ksw(b), want)

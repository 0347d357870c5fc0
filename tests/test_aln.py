"""Chains -> alignment regions: the loop of
mem_align1_core over every read's chains (software/bwamem.c:1452-1460),
mem_chain2aln_short (software/bwamem.c:805-852, ksw_align2) and, when it
declines, mem_chain2aln (software/bwamem.c:1040-1188, ksw_extend2 both ways).

Bar: bit-exact — per read, every region's rb / re / qb / qe / score / truesc /
csub / w / seedcov in the reference's order.  The restatement
(oracle/aln_oracle.c) is pinned to the compiled reference's own regions
(tests/golden/*.smrg.gz, `ref_harness aln`) over the reference's own
filtered chains (the matching *.smch.gz); the GPU path (smem_chain2aln,
through the C ABI) is checked against the same fixtures and against the
restatement on larger repeat-rich genomes with chains from the GPU chain stage.
"""
import numpy as np
import pytest

from oracle import oracle
from tests import golden_data

FIX = golden_data.aln_fixtures()
FIELDS = ["rb", "re", "qb", "qe", "score", "truesc", "sub", "csub", "sub_n", "w", "seedcov", "secondary"]


def _reads(g, n):
    from smemgpu import synth
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        p = golden_data.files(g, d)
        return synth.read_smrd(p["smrd"]).subset(np.arange(n))


def _case_inputs(fix):
    cases = golden_data.genome_cases(fix["genome"])
    case = next(c for c in cases if c["name"] == fix["case"])
    chain = next(c for c in case["chains"] if c["file"] == fix["chain_file"])
    chains, chain_off, seeds = golden_data.smch_parse(golden_data.smch(chain))
    reads = _reads(fix["genome"], case["n_reads"])
    assert chain_off.size == reads.n + 1
    return reads, chains, chain_off, seeds


def _assert_same(got, got_off, want, want_off):
    assert np.array_equal(np.asarray(got_off, dtype=np.uint64), np.asarray(want_off, dtype=np.uint64))
    for f in FIELDS:
        bad = np.nonzero(got[f] != want[f])[0]
        assert bad.size == 0, f"field {f}: {bad.size} regions differ, first {bad[:5]}"


def test_aln_fixtures_present():
    assert len(FIX) >= 4
    assert {f["genome"] for f in FIX} == {"g1", "g2"}


@pytest.mark.parametrize("fix", FIX, ids=[f["file"].split(".")[0] for f in FIX])
def test_aln_oracle_vs_reference(fix):
    """restatement == the reference's mem_chain2aln loop, region for region"""
    reads, chains, chain_off, seeds = _case_inputs(fix)
    want, want_off = golden_data.smrg_parse(golden_data.smrg(fix))
    assert want.size > 0
    got, got_off = oracle.aln(golden_data.pac(fix["genome"]), golden_data.l_pac(fix["genome"]), reads.codes,
                              reads.offs, chains, chain_off, seeds,
                              oracle.aln_opt(w=fix["w"], min_seed_len=fix["min_seed_len"]))
    _assert_same(got, got_off, want, want_off)


@pytest.mark.gpu
@pytest.mark.parametrize("heavy", [None, "1", "1000:2", "1+nocand"],
                         ids=["default", "all_heavy", "seed_heavy", "all_heavy_bin_hash"])
@pytest.mark.parametrize("fix", FIX, ids=[f["file"].split(".")[0] for f in FIX])
def test_aln_gpu_vs_reference(gpu_device, fix, heavy, monkeypatch):
    """heavy = "1": every read takes the heavy-read path (regions computed
    ahead per chain, then the read's walk), SMEM_ALN_HEAVY_MIN."""
    _heavy_env(monkeypatch, heavy)
    import smemgpu
    from smemgpu import synth
    reads, chains, chain_off, seeds = _case_inputs(fix)
    want, want_off = golden_data.smrg_parse(golden_data.smrg(fix))
    idx = smemgpu.Index.read(golden_data.files(fix["genome"], _tmpdir())["bwt"])
    gpu = smemgpu.Gpu(idx, device=gpu_device)
    try:
        raw, off, ms = gpu.chain2aln(golden_data.pac(fix["genome"]), golden_data.l_pac(fix["genome"]), reads.codes,
                                     reads.offs, chains, chain_off, seeds,
                                     oracle.aln_opt(w=fix["w"], min_seed_len=fix["min_seed_len"]))
    finally:
        gpu.close()
    got = np.frombuffer(raw.tobytes(), dtype=golden_data.ALNREG_DT)
    _assert_same(got, off, want, want_off)
    del synth


def _heavy_env(monkeypatch, heavy):
    """heavy = "min[:seeds]": SMEM_ALN_HEAVY_MIN / SMEM_ALN_HEAVY_SEEDS, the
    chain / seed counts from which a read takes the heavy-read path; its walk
    then tests containment through the candidate index, or, with "+nocand"
    (SMEM_ALN_CAND=0), always through the region bin hash (SMEM_ALN_HASH_MIN
    = 1).  A "/1"
    suffix: the light and heavy reads' kernels one after the other on the
    batch's stream (SMEM_ALN_STREAMS=1) instead of side by side."""
    while heavy and "+" in heavy:
        heavy, _, opt = heavy.rpartition("+")
        if opt == "inline":
            # the heavy-read walk inlined into its kernel (the round-2 hang's
            # shape), every loop iteration counted against a guard: a walk that
            # would spin fails the call instead of hanging
            monkeypatch.setenv("SMEM_ALN_WALK_INLINE", "1")
        elif opt == "nolane":
            # no regions computed ahead one seed per lane (SMEM_ALN_LANE=0)
            monkeypatch.setenv("SMEM_ALN_LANE", "0")
        elif opt == "nocand":
            # the heavy walk without the candidate index (the bin hash of the
            # regions made so far)
            monkeypatch.setenv("SMEM_ALN_CAND", "0")
        elif opt.startswith("giants"):
            # the giant split's size (SMEM_ALN_GIANTS; 0: off): the heaviest heavy reads'
            # passes, candidate index and walk on the batch's third stream
            monkeypatch.setenv("SMEM_ALN_GIANTS", opt[len("giants"):])
        elif opt.startswith("gfirst"):
            # whose passes wait for the giants' (SMEM_ALN_GIANT_FIRST 0 / 1 / 2)
            monkeypatch.setenv("SMEM_ALN_GIANT_FIRST", opt[len("gfirst"):])
    if heavy and "/" in heavy:
        heavy, _, streams = heavy.partition("/")
        monkeypatch.setenv("SMEM_ALN_STREAMS", streams)
    if heavy:
        m, _, sd = heavy.partition(":")
        monkeypatch.setenv("SMEM_ALN_HEAVY_MIN", m)
        if sd:
            monkeypatch.setenv("SMEM_ALN_HEAVY_SEEDS", sd)
        monkeypatch.setenv("SMEM_ALN_HASH_MIN", "1")  # every heavy walk through the bin hash


def _tmpdir():
    import tempfile
    return tempfile.mkdtemp()


def _pack(codes):
    """2-bit forward strand as bns_fasta2bntseq packs it (software/bntseq.c:303-309)"""
    c = np.asarray(codes, dtype=np.uint8)
    c = np.where(c > 3, 0, c).astype(np.uint8)
    pad = (-c.size) % 4
    c = np.concatenate([c, np.zeros(pad, dtype=np.uint8)]).reshape(-1, 4)
    return (c[:, 0] << 6 | c[:, 1] << 4 | c[:, 2] << 2 | c[:, 3]).astype(np.uint8)


def test_pack_matches_reference_pac():
    """the test-side packer gives bwa_index's .pac on the golden genomes (no N)"""
    import gzip
    import os
    for g in ("g1", "g2"):
        with gzip.open(os.path.join(golden_data.GOLDEN, g + ".fa.gz"), "rb") as fh:
            codes = golden_data.fasta_codes(fh.read())
        assert np.array_equal(_pack(codes), golden_data.pac(g))


@pytest.mark.gpu
@pytest.mark.parametrize("w,a,heavy", [(100, 1, None), (20, 1, None), (100, 2, None), (100, 1, "1"), (100, 2, "1"),
                                       (20, 1, "3"), (100, 1, "0"), (100, 1, "1000:3"), (100, 1, "3/1"),
                                       (100, 1, "1+inline"), (100, 2, "3+inline"), (100, 1, "0+nolane"),
                                       (100, 1, "1+nolane"), (100, 2, "3+nolane"), (100, 1, "1+nocand"),
                                       (100, 2, "3+nocand"), (100, 1, "1+giants0"), (100, 1, "1+giants7"),
                                       (100, 2, "3+giants64+gfirst0"), (100, 1, "1+giants100000+gfirst1")])
def test_aln_gpu_vs_oracle_repeat_dense(gpu_device, w, a, heavy, monkeypatch):
    """600 kbp, 60 % diverged repeat copies; 4000 reads of 70..700 bp (both
    kernel instantiations) with substitutions and Ns; chains from the GPU
    chain stage; GPU regions == restatement, through the host API
    (smem_chain2aln, explicit .pac and resident .pac) and the device-resident
    batch stage (smem_batch_chain2aln over the chains left in HBM).  a = 2
    (-A 2 scaling, b 8, gaps 12 + 2) sends the short path's longer queries
    through ksw_align2's 16-bit branch.  heavy: SMEM_ALN_HEAVY_MIN (1: every
    read through the heavy-read path, 3: reads with 3+ chains, 0: none,
    1000:3 reads with 3+ seeds); giants<N>: the giant split's size (0: off,
    100000: every heavy read), gfirst<K>: whose passes wait for the giants'."""
    _heavy_env(monkeypatch, heavy)
    import smemgpu
    from smemgpu import synth
    g = synth.make_genome(600_000, seed=91, repeat_frac=0.6, n_families=5, exact_frac=0.01, tandem_frac=0.01)
    idx, sa = smemgpu.Index.build_sa(g.codes, sa_intv=32)
    gpu = smemgpu.Gpu(idx, device=gpu_device)
    try:
        gpu.load_sa(sa)
        reads = synth.concat_reads([synth.make_reads(g.codes, 2000, 150, seed=92, sub_rate=0.02),
                                    synth.make_reads(g.codes, 1000, (70, 250), seed=93, n_rate=0.01, sub_rate=0.03),
                                    synth.make_reads(g.codes, 600, (257, 700), seed=94, sub_rate=0.02),
                                    synth.make_reads(g.codes, 400, 101, seed=95, random_frac=0.3)])
        opt = oracle.aln_opt(w=w) if a == 1 else oracle.aln_opt(w=w, a=2, b=8, o_del=12, e_del=2, o_ins=12, e_ins=2)
        pac = _pack(g.codes)
        l_pac = int(g.codes.size)
        gpu.load_pac(pac, l_pac)
        b = gpu.batch(reads.n, reads.codes.size, int(reads.lens.max()))
        try:
            b.set_reads(reads.codes, reads.offs)
            b.run(smemgpu.Options())
            b.sa(19, 10000)
            b.chain(l_pac, w=w)
            b.chain2aln(opt)   # device-resident: chains, seeds, reads and .pac already in HBM
            res = b.fetch()
            chains, chain_off, seeds = res.chains, res.chain_off, res.seeds
            assert b.stats()["n_regs"] == int(res.reg_off[-1])
        finally:
            b.close()
        raw, off, ms = gpu.chain2aln(pac, l_pac, reads.codes, reads.offs, chains, chain_off, seeds, opt)
        raw2, off2, _ = gpu.chain2aln(None, l_pac, reads.codes, reads.offs, chains, chain_off, seeds, opt)
    finally:
        gpu.close()
    want, want_off = oracle.aln(pac, l_pac, reads.codes, reads.offs, chains, chain_off, seeds, opt)
    assert want.size > 1000
    for r, o in ((raw, off), (raw2, off2), (res.regs, res.reg_off)):
        got = np.frombuffer(r.tobytes(), dtype=golden_data.ALNREG_DT)
        _assert_same(got, o, want, want_off)


@pytest.mark.gpu
def test_aln_gpu_argument_checks(gpu_device):
    """The host API refuses query codes > 4 (they would index past the scoring
    matrix), chains sharing seeds (they would share sort scratch), a short
    .pac and a missing resident .pac; the batch stage needs filtered chains."""
    import smemgpu
    from smemgpu import synth
    g = synth.make_genome(50_000, seed=3)
    idx, sa = smemgpu.Index.build_sa(g.codes, sa_intv=32)
    gpu = smemgpu.Gpu(idx, device=gpu_device)
    try:
        gpu.load_sa(sa)
        reads = synth.make_reads(g.codes, 50, 150, seed=4)
        b = gpu.batch(reads.n, reads.codes.size, 150)
        b.set_reads(reads.codes, reads.offs)
        b.run()
        b.sa(19, 10000)
        b.chain(g.codes.size, filter=False)
        with pytest.raises(smemgpu.SmemError):   # unfiltered chains
            b.chain2aln(oracle.aln_opt())
        b.chain(g.codes.size)
        with pytest.raises(smemgpu.SmemError):   # no resident .pac
            b.chain2aln(oracle.aln_opt())
        res = b.fetch()
        b.close()
        opt = oracle.aln_opt()
        pac = _pack(g.codes)
        l_pac = int(g.codes.size)
        with pytest.raises(smemgpu.SmemError):   # no pac given, none resident
            gpu.chain2aln(None, l_pac, reads.codes, reads.offs, res.chains, res.chain_off, res.seeds, opt)
        with pytest.raises(smemgpu.SmemError):   # short pac
            gpu.chain2aln(pac[:10], l_pac, reads.codes, reads.offs, res.chains, res.chain_off, res.seeds, opt)
        bad = reads.codes.copy()
        bad[5] = 7
        with pytest.raises(smemgpu.SmemError):   # code > 4
            gpu.chain2aln(pac, l_pac, bad, reads.offs, res.chains, res.chain_off, res.seeds, opt)
        ch = res.chains.copy()
        k = int(np.nonzero(ch["n"] > 0)[0][1])
        ch["seed_off"][k] = ch["seed_off"][int(np.nonzero(ch["n"] > 0)[0][0])]
        with pytest.raises(smemgpu.SmemError):   # chains sharing seeds
            gpu.chain2aln(pac, l_pac, reads.codes, reads.offs, ch, res.chain_off, res.seeds, opt)
    finally:
        gpu.close()

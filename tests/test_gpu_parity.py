"""GPU parity: the HIP seeding path (through the C ABI) against the oracle.

Bar: bit-exact — every interval list smem_next2 would return, in order
(SURVEY.md §8(b) parity unit).  Cases cover the edge cases the reference's
code paths have: ambiguous bases (software/bwt.c:800-803, bwamem.c:252),
reads shorter than the seed length (bwamem.c:600), split_len = len
(bwamem.c:458), -e start width 2 (bwamem.c:457), re-seeding and the ordered
merge (bwamem.c:272-301), multi-occurrence / tandem intervals, random
reads, output-capacity overflow, empty batches, and concurrent host workers.
"""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

OPTS = {
    "default": dict(min_seed_len=19, split_factor=1.5, split_width=10, start_width=1),
    "noexact": dict(min_seed_len=19, split_factor=1.5, split_width=10, start_width=2),
    "k14s20": dict(min_seed_len=14, split_factor=1.5, split_width=20, start_width=1),
    "reseed": dict(min_seed_len=19, split_factor=1.0, split_width=500, start_width=1),
    "k30": dict(min_seed_len=30, split_factor=2.0, split_width=3, start_width=1),
}


@pytest.fixture(scope="module")
def world(gpu_device):
    import smemgpu
    from smemgpu import synth
    genome = synth.make_genome(400_000, seed=21)
    idx = smemgpu.Index.build(genome.codes)
    gpu = smemgpu.Gpu(idx, device=gpu_device)
    ref = oracle.OracleIndex(words=idx.words, primary=idx.primary, L2=idx.L2)
    yield dict(genome=genome, idx=idx, gpu=gpu, ref=ref)
    gpu.close()


def _reads(genome, kind, seed):
    from smemgpu import synth
    g = genome.codes
    if kind == "150bp":
        return synth.make_reads(g, 2000, 150, seed=seed)
    if kind == "mixed":
        return synth.concat_reads([
            synth.make_reads(g, 500, (1, 320), seed=seed, n_rate=0.02),
            synth.make_reads(g, 200, (15, 40), seed=seed + 1),
            synth.make_reads(g, 200, 101, seed=seed + 2, sub_rate=0.05, random_frac=0.3),
        ])
    if kind == "250bp5":
        return synth.make_reads(g, 800, 250, seed=seed, sub_rate=0.05)
    raise ValueError(kind)


def _compare(world, reads, opt, **gpu_kw):
    import smemgpu
    want, per, st = oracle.seed(world["ref"], reads.codes, reads.offs, threads=4, **opt)
    res = smemgpu.seed(world["gpu"], reads.codes, reads.offs, smemgpu.Options(**opt))
    got = res.to_smgo()
    if got != want:
        from smemgpu import synth
        a, b = synth.read_smgo(got), synth.read_smgo(want)
        bad = [i for i in range(len(b)) if len(a[i]) != len(b[i]) or any(
            x.shape != y.shape or (x != y).any() for x, y in zip(a[i], b[i]))]
        pytest.fail(f"{len(bad)} reads differ, first {bad[:5]}")
    return st


@pytest.mark.parametrize("kind", ["150bp", "mixed", "250bp5"])
@pytest.mark.parametrize("optname", list(OPTS))
def test_parity_vs_oracle(world, kind, optname):
    reads = _reads(world["genome"], kind, seed=100 + len(optname))
    st = _compare(world, reads, OPTS[optname])
    assert st["n_intv"] > 0


def test_parity_golden_fixture(gpu_device):
    """GPU vs the compiled reference's own output on the committed fixture."""
    import smemgpu
    from smemgpu import synth
    from tests import golden_data
    fx = golden_data.load()
    gpu = smemgpu.Gpu(fx.index, device=gpu_device)
    try:
        for case in fx.cases:
            reads = fx.reads.subset(np.arange(case["n_reads"]))
            res = smemgpu.seed(gpu, reads.codes, reads.offs, smemgpu.Options(**case["opt"]))
            assert res.to_smgo() == fx.stream(case), case["name"]
    finally:
        gpu.close()


def test_edge_cases(world):
    from smemgpu import synth
    g = world["genome"].codes
    parts = []
    lens = [0, 1, 2, 18, 19, 20, 28, 29, 30, 31]
    for L in lens:
        parts.append(synth.Reads(np.array([L], np.int32), g[1000:1000 + L].copy(),
                                 np.array([0, L], np.int64)))
    # all-N, N at both ends, alternating Ns, poly-A
    for arr in (np.full(60, 4, np.uint8), np.concatenate([[4], g[5000:5100], [4]]).astype(np.uint8),
                np.where(np.arange(120) % 7 == 0, 4, g[9000:9120]).astype(np.uint8), np.zeros(150, np.uint8)):
        parts.append(synth.Reads(np.array([arr.size], np.int32), arr, np.array([0, arr.size], np.int64)))
    reads = synth.concat_reads(parts)
    for opt in OPTS.values():
        _compare(world, reads, opt)


def test_empty_batch(world):
    import smemgpu
    res = smemgpu.seed(world["gpu"], np.zeros(0, np.uint8), np.zeros(1, np.uint64))
    assert res.intv.shape == (0, 4)
    assert res.intv_off.tolist() == [0]


def test_overflow_pass(world, gpu_device):
    """Tiny per-read output capacity forces the overflow re-run path."""
    import smemgpu
    from smemgpu import synth
    gpu = smemgpu.Gpu(world["idx"], device=gpu_device, intv_cap=2)
    try:
        reads = _reads(world["genome"], "mixed", seed=7)
        want, _, _ = oracle.seed(world["ref"], reads.codes, reads.offs, threads=4)
        b = gpu.batch(reads.n, reads.codes.size, int(reads.lens.max()))
        b.set_reads(reads.codes, reads.offs)
        b.run()
        assert b.stats()["n_overflow"] > 0
        assert b.fetch().to_smgo() == want
        b.close()
    finally:
        gpu.close()


def test_few_lanes_many_reads_per_lane(world, gpu_device):
    import smemgpu
    gpu = smemgpu.Gpu(world["idx"], device=gpu_device, lanes_per_cu=64)
    try:
        reads = _reads(world["genome"], "150bp", seed=9)
        want, _, _ = oracle.seed(world["ref"], reads.codes, reads.offs, threads=4)
        assert smemgpu.seed(gpu, reads.codes, reads.offs).to_smgo() == want
    finally:
        gpu.close()


@pytest.mark.parametrize("variant", [3, 4, 5, 6, 9, 10, 11, 12, 13, 16, 19, 20, 21, 22, 24, 25, 27, 28, 29, 30, 31])
def test_kernel_variants(world, gpu_device, variant):
    """The A/B builds (reference-layout fetches, stamped, forward-list LDS
    ring) are bit-exact too.  The product library instantiates 9 (stamped)
    and 20 (= the default); the others need a library built with
    `make -C bwa-mem-harp2_amd AB=1` (lib_ab/, run with SMEMGPU_LIB)."""
    import smemgpu
    if not smemgpu.load().smem_seed_variant_built(variant):
        pytest.skip(f"A/B variant {variant} is not in this build (make AB=1)")
    gpu = smemgpu.Gpu(world["idx"], device=gpu_device, variant=variant)
    try:
        reads = synth_concat(_reads(world["genome"], "mixed", seed=11), _reads(world["genome"], "250bp5", seed=12))
        for opt in ((OPTS["default"], OPTS["reseed"]) if variant < 11 else OPTS.values()):
            want, _, _ = oracle.seed(world["ref"], reads.codes, reads.offs, threads=4, **opt)
            assert smemgpu.seed(gpu, reads.codes, reads.offs, smemgpu.Options(**opt)).to_smgo() == want
    finally:
        gpu.close()


WP_VARIANTS = [40, 41, 42, 43, 44, 45, 46, 47, 48, 49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60, 61, 62]


def _need_variant(variant):
    """The product library instantiates the default (49) and its k-mer twin
    (54) only; the other A/B variants need `make AB=1` (SMEMGPU_LIB)."""
    import smemgpu
    if not smemgpu.load().smem_seed_variant_built(variant):
        pytest.skip(f"A/B variant {variant} is not in this build (make AB=1)")


def _edge_reads(g):
    from smemgpu import synth
    parts = []
    for L in [0, 1, 2, 18, 19, 20, 28, 29, 30, 31]:
        parts.append(synth.Reads(np.array([L], np.int32), g[1000:1000 + L].copy(), np.array([0, L], np.int64)))
    for arr in (np.full(60, 4, np.uint8), np.concatenate([[4], g[5000:5100], [4]]).astype(np.uint8),
                np.where(np.arange(120) % 7 == 0, 4, g[9000:9120]).astype(np.uint8), np.zeros(150, np.uint8)):
        parts.append(synth.Reads(np.array([arr.size], np.int32), arr, np.array([0, arr.size], np.int64)))
    return synth.concat_reads(parts)


@pytest.mark.parametrize("variant", WP_VARIANTS)
def test_wp_kernel_parity(world, gpu_device, variant):
    """seed_wp_kernel (variants 40-43: owners per wave x LDS list entries x
    wave priority): the backward steps' entries extended by the whole wave,
    pruned by ballots (software/bwt.c:812-826) -- bit-exact against the
    oracle on every read kind and option set, the edge cases, the overflow
    pass and a grid with fewer lanes than reads."""
    import smemgpu
    _need_variant(variant)
    gpu = smemgpu.Gpu(world["idx"], device=gpu_device, variant=variant)
    try:
        g = world["genome"].codes
        for kind in ("150bp", "mixed", "250bp5"):
            reads = _reads(world["genome"], kind, seed=300 + variant)
            for opt in OPTS.values():
                want, _, _ = oracle.seed(world["ref"], reads.codes, reads.offs, threads=4, **opt)
                got = smemgpu.seed(gpu, reads.codes, reads.offs, smemgpu.Options(**opt)).to_smgo()
                assert got == want, (kind, opt)
        edge = _edge_reads(g)
        for opt in OPTS.values():
            want, _, _ = oracle.seed(world["ref"], edge.codes, edge.offs, threads=4, **opt)
            assert smemgpu.seed(gpu, edge.codes, edge.offs, smemgpu.Options(**opt)).to_smgo() == want, opt
    finally:
        gpu.close()
    reads = _reads(world["genome"], "mixed", seed=7)
    want, _, _ = oracle.seed(world["ref"], reads.codes, reads.offs, threads=4)
    gpu = smemgpu.Gpu(world["idx"], device=gpu_device, variant=variant, intv_cap=2)
    try:  # the overflow pass
        b = gpu.batch(reads.n, reads.codes.size, int(reads.lens.max()))
        b.set_reads(reads.codes, reads.offs)
        b.run()
        assert b.stats()["n_overflow"] > 0
        assert b.fetch().to_smgo() == want
        b.close()
    finally:
        gpu.close()
    gpu = smemgpu.Gpu(world["idx"], device=gpu_device, variant=variant, lanes_per_cu=64)
    try:  # many reads per owner
        assert smemgpu.seed(gpu, reads.codes, reads.offs).to_smgo() == want
    finally:
        gpu.close()


@pytest.mark.parametrize("variant,k", [(54, 1), (54, 7), (54, 11), (55, 12), (55, 2), (57, 11)])
def test_wp_kmer_table(world, gpu_device, variant, k):
    """seed_wp_kernel with the k-mer table (variants 54, 55): forward and
    backward extends whose result has <= k bases read the table; every read
    kind and option set bit-exact against the oracle."""
    import smemgpu
    _need_variant(variant)
    gpu = smemgpu.Gpu(world["idx"], device=gpu_device, variant=variant, kmer_k=k)
    try:
        reads = synth_concat(_reads(world["genome"], "mixed", seed=13), _reads(world["genome"], "250bp5", seed=14))
        for opt in OPTS.values():
            want, _, _ = oracle.seed(world["ref"], reads.codes, reads.offs, threads=4, **opt)
            assert smemgpu.seed(gpu, reads.codes, reads.offs, smemgpu.Options(**opt)).to_smgo() == want, opt
    finally:
        gpu.close()


@pytest.mark.parametrize("k", [1, 2, 7, 10, 12])
def test_kmer_table_variant(world, gpu_device, k):
    """Variant 23: extends whose result has <= k bases read the k-mer table;
    the lists must be the oracle's bit for bit (a bi-interval does not depend
    on the extension path), edge-case reads included."""
    import smemgpu
    from smemgpu import synth
    _need_variant(23)
    gpu = smemgpu.Gpu(world["idx"], device=gpu_device, variant=23, kmer_k=k)
    try:
        g = world["genome"].codes
        edge = synth.Reads(np.array([120], np.int32), np.where(np.arange(120) % 7 == 0, 4, g[9000:9120]).astype(np.uint8),
                           np.array([0, 120], np.int64))
        reads = synth_concat(_reads(world["genome"], "mixed", seed=13), _reads(world["genome"], "250bp5", seed=14), edge)
        for opt in OPTS.values():
            want, _, _ = oracle.seed(world["ref"], reads.codes, reads.offs, threads=4, **opt)
            assert smemgpu.seed(gpu, reads.codes, reads.offs, smemgpu.Options(**opt)).to_smgo() == want
    finally:
        gpu.close()


def test_kmer_table_arguments(world, gpu_device):
    import smemgpu
    _need_variant(23)
    gpu = smemgpu.Gpu(world["idx"], device=gpu_device, variant=23)
    try:
        reads = _reads(world["genome"], "150bp", seed=15)
        with pytest.raises(RuntimeError, match="kmer"):
            smemgpu.seed(gpu, reads.codes, reads.offs)
        for bad in (-1, 16):
            with pytest.raises(RuntimeError):
                gpu.set_kmer_table(bad)
        gpu.set_kmer_table(6)
        gpu.set_kmer_table(9)  # rebuilt in place
        want, _, _ = oracle.seed(world["ref"], reads.codes, reads.offs, threads=4)
        assert smemgpu.seed(gpu, reads.codes, reads.offs).to_smgo() == want
        gpu.set_kmer_table(0)
        with pytest.raises(RuntimeError, match="kmer"):
            smemgpu.seed(gpu, reads.codes, reads.offs)
    finally:
        gpu.close()


def synth_concat(*parts):
    from smemgpu import synth
    return synth.concat_reads(list(parts))


def test_batch_reuse(world):
    """One batch object, several runs with different reads (no stale state)."""
    from smemgpu import synth
    g = world["genome"].codes
    r1 = synth.make_reads(g, 700, 150, seed=31)
    r2 = synth.make_reads(g, 300, (20, 150), seed=32, n_rate=0.01)
    b = world["gpu"].batch(1000, 200_000, 150)
    for r in (r1, r2, r1):
        want, _, _ = oracle.seed(world["ref"], r.codes, r.offs, threads=4)
        b.set_reads(r.codes, r.offs)
        b.run()
        assert b.fetch().to_smgo() == want
    b.close()


def test_host_driver_threads(world, tmp_path):
    """The C host driver (kt_for_batch workers calling smem_gpu_collect
    concurrently) writes the same stream as the oracle."""
    from smemgpu import synth
    from smemgpu.lib import PKG_DIR
    reads = _reads(world["genome"], "mixed", seed=41)
    bwt = str(tmp_path / "g.bwt")
    world["idx"].write(bwt)
    smrd = str(tmp_path / "r.smrd")
    synth.write_smrd(smrd, reads)
    out = str(tmp_path / "o.smgo")
    exe = os.path.join(PKG_DIR, "bin", "smem_seed")
    subprocess.run([exe, "-t", "4", "-b", "97", bwt, smrd, out], check=True, timeout=300)
    want, _, _ = oracle.seed(world["ref"], reads.codes, reads.offs, threads=4)
    with open(out, "rb") as fh:
        assert fh.read() == want


@pytest.mark.parametrize("n_bp,seed", [(1, 1), (7, 2), (64, 3), (1000, 4), (4099, 5), (250_000, 6)])
def test_gpu_index_builder_matches_cpu(gpu_device, n_bp, seed):
    """smem_bwt_build_gpu (prefix doubling) == smem_bwt_build (SA-IS) byte for byte;
    the CPU builder is itself pinned to `bwa index -a is` (tests/test_oracle.py)."""
    import smemgpu
    from smemgpu import synth
    g = synth.make_genome(n_bp, seed=seed, n_chrom=1)
    a = smemgpu.Index.build(g.codes)
    b = smemgpu.Index.build_gpu(g.codes, device=gpu_device)
    assert a.primary == b.primary and a.L2.tolist() == b.L2.tolist()
    assert np.array_equal(a.words, b.words)


@pytest.mark.parametrize("kind,n_bp", [("rand", 1), ("rand", 7), ("rand", 64), ("rand", 4099), ("rand", 250_000),
                                       ("rand", 3_000_000), ("polyA", 20_000), ("tandem3", 30_000),
                                       ("dup", 200_000)])
def test_gpu_large_builder_matches_cpu(gpu_device, kind, n_bp):
    """The bucketed 64-bit builder (human-size genomes) == SA-IS byte for byte,
    .bwt and .sa, forced at small sizes; repeat-only genomes drive its doubling
    phase through many rounds over nearly every suffix."""
    import smemgpu
    from smemgpu import synth
    if kind == "rand":
        g = synth.make_genome(n_bp, seed=n_bp % 97, n_chrom=1).codes
    elif kind == "polyA":
        g = np.zeros(n_bp, dtype=np.uint8)
    elif kind == "tandem3":
        g = np.resize(np.array([0, 1, 3], dtype=np.uint8), n_bp)
        g[n_bp // 2] = 2
    else:  # a random genome written twice, then a third copy with one change
        h = np.random.default_rng(3).integers(0, 4, n_bp // 3, dtype=np.uint8)
        g = np.concatenate([h, h, h])
        g[-5] = (g[-5] + 1) & 3
    a_idx, a_sa = smemgpu.Index.build_sa(g, sa_intv=32)
    b_idx, b_sa = smemgpu.Index.build_sa(g, sa_intv=32, gpu=True, device=gpu_device, large=True)
    assert a_idx.primary == b_idx.primary and a_idx.L2.tolist() == b_idx.L2.tolist()
    assert np.array_equal(a_idx.words, b_idx.words)
    assert np.array_equal(a_sa.samples, b_sa.samples)
    c = smemgpu.Index.build_gpu(g, device=gpu_device, large=True)
    assert np.array_equal(a_idx.words, c.words)


@pytest.mark.parametrize("sb_max", ["1000", "65536"])
def test_gpu_large_builder_many_superbuckets(gpu_device, monkeypatch, sb_max):
    """The bucketed builder with its super-buckets shrunk (the human-size
    genome has ~25 of 2^28 suffixes): every bin's range is sorted on its own
    and the ranks / unresolved list are carried across them."""
    import smemgpu
    from smemgpu import synth
    monkeypatch.setenv("SMEM_BUILD_SB_MAX", sb_max)
    g = synth.make_genome(1_500_000, seed=61, n_chrom=1).codes
    a_idx, a_sa = smemgpu.Index.build_sa(g, sa_intv=32)
    b_idx, b_sa = smemgpu.Index.build_sa(g, sa_intv=32, gpu=True, device=gpu_device, large=True)
    assert a_idx.primary == b_idx.primary and np.array_equal(a_idx.words, b_idx.words)
    assert np.array_equal(a_sa.samples, b_sa.samples)


def test_gpu_index_builder_golden(gpu_device):
    import smemgpu
    from tests import golden_data
    fx = golden_data.load()
    b = smemgpu.Index.build_gpu(fx.genome, device=gpu_device)
    assert b.primary == fx.index.primary
    assert np.array_equal(b.words, fx.index.words)


# ---------------------------------------------------------------- bwt_sa
def test_sa_golden_fixture(gpu_device, tmp_path):
    """GPU bwt_sa of every seed occurrence == the reference's (golden SMSA)."""
    import smemgpu
    from tests import golden_data
    fx = golden_data.load()
    p = str(tmp_path / "g1.sa")
    with open(p, "wb") as fh:
        fh.write(fx.sa_bytes)
    sa = smemgpu.SA.read(p)
    gpu = smemgpu.Gpu(fx.index, device=gpu_device)
    try:
        gpu.load_sa(sa)
        for case in fx.cases:
            reads = fx.reads.subset(np.arange(case["n_reads"]))
            b = gpu.batch(reads.n, reads.codes.size, int(reads.lens.max()))
            b.set_reads(reads.codes, reads.offs)
            b.run(smemgpu.Options(**case["opt"]))
            b.sa(case["opt"]["min_seed_len"], case["max_occ"])
            res = b.fetch()
            assert res.to_smgo() == fx.stream(case), case["name"]
            assert res.to_smsa() == fx.sa_stream(case), case["name"]
            assert b.stats()["n_occ"] == case["n_occ"]
            b.close()
    finally:
        gpu.close()


@pytest.mark.parametrize("densify", ["hop", "walk", "raw"])
@pytest.mark.parametrize("max_occ", [1, 20, 10000])
def test_sa_vs_oracle(gpu_device, max_occ, densify, monkeypatch):
    """Random genome with repeats, mixed reads: GPU positions == restated bwt_sa
    (the device SA densified by hop + chase passes, or by one walk per row, or
    the walk to the uploaded samples -- what the lookups use while the
    densification still runs)."""
    if densify == "raw":
        monkeypatch.setenv("SMEM_GPU_SA_RAW", "1")
    else:
        monkeypatch.setenv("SMEM_GPU_DENSIFY", densify)
    import smemgpu
    from smemgpu import synth
    g = synth.make_genome(300_000, seed=41)
    idx, sa = smemgpu.Index.build_sa(g.codes, sa_intv=32)
    gpu = smemgpu.Gpu(idx, device=gpu_device)
    oidx = oracle.OracleIndex(words=idx.words, primary=idx.primary, L2=idx.L2)
    osa = oracle.OracleSA(sa=sa.samples, sa_intv=32, seq_len=idx.seq_len)
    try:
        gpu.load_sa(sa)
        reads = _reads(g, "mixed", seed=43)
        b = gpu.batch(reads.n, reads.codes.size, int(reads.lens.max()))
        b.set_reads(reads.codes, reads.offs)
        b.run()
        b.sa(19, max_occ)
        res = b.fetch()
        counts, k = oracle.sa_queries([res.read_calls(i) for i in range(reads.n)], 19, max_occ)
        assert np.array_equal(res.sa_pos, osa.lookup(oidx, k))
        assert [res.read_sa(i).size for i in range(reads.n)] == counts.tolist()
        b.close()
    finally:
        gpu.close()
        osa.close()
        oidx.close()


@pytest.mark.parametrize("densify", ["hop", "walk", "raw"])
def test_sa_intervals_and_errors(gpu_device, densify, monkeypatch):
    """Other sampling intervals; SA of another index rejected; sa before run rejected."""
    if densify == "raw":
        monkeypatch.setenv("SMEM_GPU_SA_RAW", "1")
    else:
        monkeypatch.setenv("SMEM_GPU_DENSIFY", densify)
    import smemgpu
    from smemgpu import synth
    g = synth.make_genome(50_000, seed=45)
    reads = synth.make_reads(g.codes, 400, 150, seed=46)
    for intv in (1, 8, 128):
        idx, sa = smemgpu.Index.build_sa(g.codes, sa_intv=intv)
        gpu = smemgpu.Gpu(idx, device=gpu_device)
        oidx = oracle.OracleIndex(words=idx.words, primary=idx.primary, L2=idx.L2)
        osa = oracle.OracleSA(sa=sa.samples, sa_intv=intv, seq_len=idx.seq_len)
        gpu.load_sa(sa)
        b = gpu.batch(reads.n, reads.codes.size, 150)
        with pytest.raises(smemgpu.SmemError):
            b.sa()
        b.set_reads(reads.codes, reads.offs)
        b.run()
        b.sa()
        res = b.fetch()
        _, k = oracle.sa_queries([res.read_calls(i) for i in range(reads.n)])
        assert np.array_equal(res.sa_pos, osa.lookup(oidx, k)), intv
        b.close()
        gpu.close()
        osa.close()
        oidx.close()
    other_idx, other_sa = smemgpu.Index.build_sa(synth.make_genome(50_001, seed=47).codes)
    idx = smemgpu.Index.build(g.codes)
    gpu = smemgpu.Gpu(idx, device=gpu_device)
    with pytest.raises(smemgpu.SmemError):
        gpu.load_sa(other_sa)
    gpu.close()


@pytest.mark.parametrize("n_bp", [3000, 250_000])
def test_gpu_builder_sa_matches_cpu(gpu_device, n_bp):
    import smemgpu
    from smemgpu import synth
    g = synth.make_genome(n_bp, seed=48).codes
    a_idx, a_sa = smemgpu.Index.build_sa(g, sa_intv=32)
    b_idx, b_sa = smemgpu.Index.build_sa(g, sa_intv=32, gpu=True, device=gpu_device)
    assert np.array_equal(a_idx.words, b_idx.words) and a_idx.primary == b_idx.primary
    assert np.array_equal(a_sa.samples, b_sa.samples)

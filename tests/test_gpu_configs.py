"""GPU parity at the BASELINE.json config sizes.

* C1: an E. coli K-12-sized genome (4,641,652 bp), 10k x 100 bp reads, 2 %
  substitutions, 0.1 % N, both strands.
* C2/C4/C5 index: a human_g1k_v37-sized genome (3,101,804,739 bp, l_pac of
  the real index: 6.2 G symbols with the reverse strand, a 3.1 GB .bwt).
  Only an index past 2^32 symbols exercises the 34-bit interval packing of
  the list entries (csrc/smem_kernels.hip PIntv), the high count bits of the
  Occ64 buckets (occ_cgt) and the 32-bit byte offsets into a 3.1 GB table
  (boff); these tests assert that intervals with x0 or x1 >= 2^32 actually
  occur in the sample.

Bar: bit-exact against the C restatement (oracle/, pinned to the compiled
reference's own streams), through the C ABI.  Reference loop:
software/bwamem.c:453-460 -> software/bwt.c:776-835; bwt_sa
software/bwt.c:104-114.
"""
import time

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

HUMAN_BP = 3_101_804_739   # human_g1k_v37 l_pac
ECOLI_BP = 4_641_652       # E. coli K-12 MG1655


def _diff(got: bytes, want: bytes) -> str:
    from smemgpu import synth
    a, b = synth.read_smgo(got), synth.read_smgo(want)
    bad = [i for i in range(len(b)) if len(a[i]) != len(b[i]) or any(
        x.shape != y.shape or (x != y).any() for x, y in zip(a[i], b[i]))]
    return f"{len(bad)} reads differ, first {bad[:5]}"


def _seed_and_compare(gpu, oidx, reads, opt: dict):
    import smemgpu
    want, _, st = oracle.seed(oidx, reads.codes, reads.offs, threads=16, **opt)
    b = gpu.batch(reads.n, int(reads.codes.size), int(reads.lens.max()))
    try:
        b.set_reads(reads.codes, reads.offs)
        b.run(smemgpu.Options(**opt))
        res = b.fetch()
    finally:
        b.close()
    got = res.to_smgo()
    assert got == want, _diff(got, want)
    return res, st


def test_c1_ecoli_sized(gpu_device):
    """BASELINE configs[0] shape: 4.64 Mbp index, 10k x 100 bp; SMEM lists and
    bwt_sa positions bit-exact."""
    import smemgpu
    from smemgpu import synth
    g = synth.make_genome(ECOLI_BP, seed=1, n_chrom=1)
    idx, sa = smemgpu.Index.build_sa(g.codes, sa_intv=32, gpu=True, device=gpu_device)
    reads = synth.make_reads(g.codes, 10_000, 100, seed=1, sub_rate=0.02, n_rate=0.001)
    oidx = oracle.OracleIndex(words=idx.words, primary=idx.primary, L2=idx.L2)
    osa = oracle.OracleSA(sa=sa.samples, sa_intv=32, seq_len=idx.seq_len)
    gpu = smemgpu.Gpu(idx, device=gpu_device)
    try:
        gpu.load_sa(sa)
        res, st = _seed_and_compare(gpu, oidx, reads, {})
        assert st["n_intv"] > 10_000
        b = gpu.batch(reads.n, int(reads.codes.size), 100)
        b.set_reads(reads.codes, reads.offs)
        b.run()
        b.sa(19, 10000)
        r2 = b.fetch()
        b.close()
        counts, k = oracle.sa_queries([r2.read_calls(i) for i in range(reads.n)], 19, 10000)
        assert np.array_equal(r2.sa_pos, osa.lookup(oidx, k))
        assert [r2.read_sa(i).size for i in range(reads.n)] == counts.tolist()
    finally:
        gpu.close()
        osa.close()
        oidx.close()


@pytest.fixture(scope="module")
def human(gpu_device):
    """The human-sized synthetic index, built once on the GPU (bucketed 64-bit
    builder), with its .sa, resident on the device."""
    import smemgpu
    from smemgpu import synth
    t = time.time()
    g = synth.make_genome(HUMAN_BP, seed=1, n_chrom=24)
    print(f"[human] genome {time.time() - t:.1f} s", flush=True)
    idx, sa = smemgpu.Index.build_sa(g.codes, sa_intv=32, gpu=True, device=gpu_device)
    print(f"[human] index {time.time() - t:.1f} s", flush=True)
    assert idx.seq_len == 2 * HUMAN_BP and idx.seq_len > 2 ** 32
    gpu = smemgpu.Gpu(idx, device=gpu_device)
    gpu.load_sa(sa)
    oidx = oracle.OracleIndex(words=idx.words, primary=idx.primary, L2=idx.L2)
    print(f"[human] ready {time.time() - t:.1f} s", flush=True)
    yield dict(codes=g.codes, idx=idx, sa=sa, gpu=gpu, oidx=oidx)
    gpu.close()
    oidx.close()


def _high_bits(res) -> int:
    x = res.intv[:, :2]
    return int(np.count_nonzero((x >> np.uint64(32)) != 0))


@pytest.mark.timeout(900)
def test_human_c2_150bp(human):
    """C2 shape: 20k x 150 bp, 2 % subs, default options, human-size index."""
    from smemgpu import synth
    reads = synth.make_reads(human["codes"], 20_000, 150, seed=2, sub_rate=0.02, n_rate=0.001)
    res, st = _seed_and_compare(human["gpu"], human["oidx"], reads, {})
    assert _high_bits(res) > 1000  # 34-bit coordinates really occur


@pytest.mark.timeout(900)
def test_human_c4_250bp(human):
    """C4 shape: 2k x 250 bp, k = 19 with re-seeding (default split options)."""
    from smemgpu import synth
    reads = synth.make_reads(human["codes"], 2_000, 250, seed=4, sub_rate=0.02, n_rate=0.001)
    res, _ = _seed_and_compare(human["gpu"], human["oidx"], reads, dict(min_seed_len=19))
    assert _high_bits(res) > 100


@pytest.mark.timeout(900)
def test_human_c5_5pct(human):
    """C5 shape: 2k x 150 bp at 5 % substitutions; also -e and re-seed-heavy options."""
    from smemgpu import synth
    reads = synth.make_reads(human["codes"], 2_000, 150, seed=5, sub_rate=0.05, n_rate=0.001)
    for opt in ({}, dict(start_width=2), dict(split_factor=1.0, split_width=500), dict(min_seed_len=14, split_width=20)):
        res, _ = _seed_and_compare(human["gpu"], human["oidx"], reads, opt)
        assert _high_bits(res) > 100


@pytest.mark.timeout(900)
def test_human_kmer_table(human, gpu_device):
    """Variant 23 with a 12-mer table at human size (34-bit table entries)."""
    import smemgpu
    from smemgpu import synth
    gpu = human["gpu"]
    if not smemgpu.load().smem_seed_variant_built(23):
        pytest.skip("A/B variant 23 is not in this build (make AB=1)")
    reads = synth.make_reads(human["codes"], 4_000, 150, seed=7, sub_rate=0.03, n_rate=0.001)
    gpu.set_kmer_table(12)
    try:
        gpu.set_variant(23)
        for opt in ({}, dict(split_factor=1.0, split_width=500)):
            res, _ = _seed_and_compare(gpu, human["oidx"], reads, opt)
            assert _high_bits(res) > 100
    finally:
        gpu.set_variant(0)
        gpu.set_kmer_table(0)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("variant", [40, 41, 49, 54])
def test_human_wp_kernel(human, variant):
    """seed_wp_kernel at human size: forward lists longer than the LDS lists
    (entries in the owner's arena, both list regions), 34-bit coordinates."""
    import smemgpu
    from smemgpu import synth
    if not smemgpu.load().smem_seed_variant_built(variant):
        pytest.skip(f"A/B variant {variant} is not in this build (make AB=1)")
    gpu = human["gpu"]
    gpu.set_variant(variant)
    if variant == 54:
        gpu.set_kmer_table(11)  # 34-bit table entries
    try:
        reads = synth.make_reads(human["codes"], 10_000, 150, seed=12, sub_rate=0.02, n_rate=0.001)
        res, _ = _seed_and_compare(gpu, human["oidx"], reads, {})
        assert _high_bits(res) > 500
        reads = synth.make_reads(human["codes"], 2_000, 250, seed=13, sub_rate=0.05, n_rate=0.001)
        for opt in ({}, dict(start_width=2), dict(split_factor=1.0, split_width=500)):
            _seed_and_compare(gpu, human["oidx"], reads, opt)
    finally:
        gpu.set_variant(0)
        gpu.set_kmer_table(0)


@pytest.mark.timeout(900)
def test_human_sa_lookup(human):
    """bwt_sa of every seed occurrence at human size (positions past 2^32)."""
    from smemgpu import synth
    reads = synth.make_reads(human["codes"], 2_000, 150, seed=6, sub_rate=0.02, n_rate=0.001)
    b = human["gpu"].batch(reads.n, int(reads.codes.size), 150)
    try:
        b.set_reads(reads.codes, reads.offs)
        b.run()
        b.sa(19, 10000)
        res = b.fetch()
    finally:
        b.close()
    osa = oracle.OracleSA(sa=human["sa"].samples, sa_intv=32, seq_len=human["idx"].seq_len)
    try:
        counts, k = oracle.sa_queries([res.read_calls(i) for i in range(reads.n)], 19, 10000)
        assert np.array_equal(res.sa_pos, osa.lookup(human["oidx"], k))
        assert [res.read_sa(i).size for i in range(reads.n)] == counts.tolist()
        assert int(np.count_nonzero(res.sa_pos >= 2 ** 32)) > 100
    finally:
        osa.close()


@pytest.mark.timeout(900)
def test_human_pe_sam_identical(human, tmp_path):
    """C3's shape at human size through the product path: 20k interleaved
    pairs (150 bp, insert N(500, 50)) on the 6.2 G-symbol index, `bwa-gpu mem
    -p -t 16` (seeding -> regions on the GPU, pairing / mate rescue / SAM on
    the CPU) against the unpatched reference pipeline (`ref_harness mem`,
    -b 1, every batch on the CPU) on the same index files: SAM byte-identical
    apart from @PG (software/fastmap.c:213-228 -> software/bwamem.c:1614)."""
    import os
    import subprocess
    from smemgpu import synth
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    bwa = os.path.join(root, "oracle", "_ref", "bwa-gpu")
    ref = os.path.join(root, "oracle", "_ref", "ref_harness")
    if not (os.path.exists(bwa) and os.path.exists(ref)):
        pytest.skip("oracle/_ref/bwa-gpu / ref_harness not built (need /root/reference at build time)")
    base = str(tmp_path / "h")
    human["idx"].write(base + ".bwt")
    human["sa"].write(base + ".sa")
    synth.write_bwa_bns(base, human["codes"])
    pe = synth.make_pairs(human["codes"], 20_000, 150, seed=11)
    fq = str(tmp_path / "p.fq")
    synth.write_fastq(fq, pe, prefix="p", pairs=True)
    sams = {}
    for name, cmd in (("gpu", [bwa, "mem", "-p", "-t", "16", "-b", "2500", base, fq]),
                      ("ref", [ref, "mem", base, fq, "16", "1", "1"])):
        p = subprocess.run(cmd, capture_output=True, timeout=600, env=dict(os.environ, SMEM_GPU_DEVICES="0"))
        err = p.stderr.decode(errors="replace")
        assert p.returncode == 0, err[-2000:]
        if name == "gpu":
            assert "seeding on the CPU" not in err and "refused" not in err, err[-2000:]
        sams[name] = [l for l in p.stdout.split(b"\n") if l and not l.startswith(b"@PG")]
    got, want = sams["gpu"], sams["ref"]
    assert len(got) == len(want) > 40_000
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    assert not bad, f"{len(bad)} SAM lines differ, first: {got[bad[0]][:200]!r} vs {want[bad[0]][:200]!r}"
    # pairs really were paired: most records carry a mate on the same contig (RNEXT "=")
    paired = sum(1 for l in got if not l.startswith(b"@") and l.split(b"\t")[6] == b"=")
    assert paired > 0.8 * 40_000

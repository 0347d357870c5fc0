"""GPU parity of the chaining stage, through the C ABI.

Bar: bit-exact — per read, the chains mem_chain returns (kbtree in-order,
software/bwamem.c:593-614) and, with the filter, what mem_chain_flt keeps
and in which order (software/bwamem.c:629-690): pos, every seed's rbeg /
qbeg / len, in order.  Checked against the compiled reference's own chains
(tests/golden/*.smch.gz: g1 and the repeat-dense g2, two option sets, both
filter modes) and against the restatement (oracle/chain_oracle.c) on larger
repeat-rich genomes: deep chain trees, duplicate chain keys, strand
bridging, long filter sorts, reads without seeds.
"""
import numpy as np
import pytest

from oracle import oracle
from tests import golden_data

pytestmark = pytest.mark.gpu

CHAINS = golden_data.chain_fixtures()


def _chain_kw(ch):
    return dict(w=ch["w"], max_chain_gap=ch["max_chain_gap"], mask_level=ch["mask_level"],
                drop_ratio=ch["drop_ratio"], filter=bool(ch["filter"]))


@pytest.fixture(scope="module")
def golden_gpus(gpu_device, tmp_path_factory):
    import smemgpu
    from smemgpu import synth
    out = {}
    for g in ("g1", "g2"):
        p = golden_data.files(g, str(tmp_path_factory.mktemp(g)))
        idx = smemgpu.Index.read(p["bwt"])
        gpu = smemgpu.Gpu(idx, device=gpu_device)
        gpu.load_sa(smemgpu.SA.read(p["sa"]))
        out[g] = (gpu, synth.read_smrd(p["smrd"]))
    yield out
    for gpu, _ in out.values():
        gpu.close()


@pytest.mark.parametrize("g,case,ch", CHAINS, ids=[c["file"].split(".")[0] for _, _, c in CHAINS])
def test_chain_golden_fixture(golden_gpus, g, case, ch):
    """GPU chains == the reference's mem_chain (+ mem_chain_flt) output."""
    import smemgpu
    gpu, reads = golden_gpus[g]
    reads = reads.subset(np.arange(case["n_reads"]))
    b = gpu.batch(reads.n, reads.codes.size, int(reads.lens.max()))
    try:
        b.set_reads(reads.codes, reads.offs)
        b.run(smemgpu.Options(**case["opt"]))
        b.sa(case["opt"]["min_seed_len"], case["max_occ"])
        b.chain(golden_data.l_pac(g), **_chain_kw(ch))
        res = b.fetch()
        assert res.to_smch() == golden_data.smch(ch)
        assert b.stats()["n_chains"] == res.chains.size
    finally:
        b.close()


def _oracle_chains(res, n_reads, l_pac, min_seed_len, max_occ, **kw):
    lists = [res.read_calls(i) for i in range(n_reads)]
    pos = [res.read_sa(i) for i in range(n_reads)]
    seeds, off = oracle.chain_seeds(lists, pos, min_seed_len, max_occ)
    return oracle.chain(seeds, off, l_pac, min_seed_len=min_seed_len, threads=8, **kw)


@pytest.mark.parametrize("opts", [
    dict(w=100, max_chain_gap=10000, mask_level=0.5, drop_ratio=0.5),
    dict(w=5, max_chain_gap=40, mask_level=0.3, drop_ratio=0.8),
    dict(w=0, max_chain_gap=1, mask_level=0.0, drop_ratio=1.0),
    dict(w=100, max_chain_gap=10000, mask_level=0.5, drop_ratio=0.0),
], ids=["std", "tight", "degenerate", "nodrop"])
@pytest.mark.parametrize("filt", [0, 1])
def test_chain_vs_oracle_repeat_dense(gpu_device, opts, filt):
    """A 1 Mbp genome that is 70 % diverged copies of 6 families plus
    tandem/exact repeats; 6000 mixed reads, max_occ 10000: hundreds of chains
    per read in places (three-level trees, long filter sorts)."""
    import smemgpu
    from smemgpu import synth
    g = synth.make_genome(1_000_000, seed=71, repeat_frac=0.7, n_families=6, exact_frac=0.02, tandem_frac=0.01)
    idx, sa = smemgpu.Index.build_sa(g.codes, sa_intv=32)
    gpu = smemgpu.Gpu(idx, device=gpu_device)
    try:
        gpu.load_sa(sa)
        reads = synth.concat_reads([synth.make_reads(g.codes, 4000, 150, seed=72, sub_rate=0.01),
                                    synth.make_reads(g.codes, 1000, (10, 300), seed=73, n_rate=0.01),
                                    synth.make_reads(g.codes, 1000, 101, seed=74, random_frac=0.3)])
        b = gpu.batch(reads.n, reads.codes.size, int(reads.lens.max()))
        b.set_reads(reads.codes, reads.offs)
        b.run()
        b.sa(19, 10000)
        l_pac = idx.seq_len // 2
        b.chain(l_pac, filter=bool(filt), **opts)
        res = b.fetch()
        want = _oracle_chains(res, reads.n, l_pac, 19, 10000, filter=filt, **opts)
        assert res.to_smch() == want
        per = [len(res.read_chains(i)) for i in range(reads.n)]
        assert max(per) > 120  # the tree splits to three levels somewhere
        b.close()
    finally:
        gpu.close()


def test_chain_strand_bridging_and_empty(gpu_device):
    """Reads across the forward/reverse boundary (seeds skipped by
    software/bwamem.c:477), reads with no seeds, and an empty batch."""
    import smemgpu
    from smemgpu import synth
    g = synth.make_genome(40_000, seed=75, n_chrom=1)
    idx, sa = smemgpu.Index.build_sa(g.codes, sa_intv=32)
    gpu = smemgpu.Gpu(idx, device=gpu_device)
    try:
        gpu.load_sa(sa)
        G = g.codes
        tail_head = np.concatenate([G[-80:], (3 - G[-80:])[::-1][:70]])  # crosses into the reverse strand
        parts = [synth.make_reads(G, 300, 150, seed=76), synth.make_reads(G, 50, 12, seed=77)]
        reads = synth.concat_reads(parts)
        codes = np.concatenate([reads.codes, tail_head.astype(np.uint8), np.zeros(0, np.uint8)])
        offs = np.concatenate([reads.offs, [reads.offs[-1] + tail_head.size, reads.offs[-1] + tail_head.size]])
        n = offs.size - 1
        b = gpu.batch(n, codes.size, 150)
        b.set_reads(codes, offs)
        b.run()
        b.sa(19, 10000)
        l_pac = idx.seq_len // 2
        for filt in (0, 1):
            b.chain(l_pac, filter=bool(filt))
            res = b.fetch()
            assert res.to_smch() == _oracle_chains(res, n, l_pac, 19, 10000, filter=filt)
        assert len(res.read_chains(n - 1)) == 0
        b.close()
        e = gpu.batch(1, 1, 1)
        e.set_reads(np.zeros(0, np.uint8), np.zeros(1, np.uint64))
        e.run()
        e.sa()
        e.chain(l_pac)
        res = e.fetch()
        assert res.chains.size == 0 and res.chain_off.tolist() == [0]
        e.close()
        f = gpu.batch(4, 600, 150)
        with pytest.raises(smemgpu.SmemError):
            f.chain(l_pac)  # before run / sa
        f.close()
    finally:
        gpu.close()


@pytest.mark.parametrize("env", [dict(SMEM_CHAIN_HEAVY_MIN="0"), dict(SMEM_CHAIN_HEAVY_MIN="100000"),
                                 dict(SMEM_CHAIN_LDS="2048"), dict(SMEM_CHAIN_TREE_ONLY="1"),
                                 dict(SMEM_CHAIN_TREE_ONLY="1", SMEM_CHAIN_HEAVY_MIN="0"),
                                 dict(SMEM_CHAIN_SERIAL_SORT="1"),
                                 dict(SMEM_CHAIN_SORT_LANE_MAX="17", SMEM_CHAIN_HEAVY_MIN="0"),
                                 dict(SMEM_CHAIN_SORT_LANE_MAX="17", SMEM_CHAIN_LDS="4096"),
                                 dict(SMEM_CHAIN_DROP_PRUNED="1", SMEM_CHAIN_HEAVY_MIN="0"),
                                 dict(SMEM_CHAIN_HEAVY_MIN="0", SMEM_CHAIN_LDS="3072"),
                                 dict(SMEM_CHAIN_STREAMS="1", SMEM_CHAIN_HEAVY_MIN="0"),
                                 dict(SMEM_CHAIN_LDS_REST="2048", SMEM_CHAIN_HEAVY_MIN="0"),
                                 dict(SMEM_CHAIN_HEAVY_MIN="0", SMEM_CHAIN_WAVE_MIN="2"),
                                 dict(SMEM_CHAIN_HEAVY_MIN="0", SMEM_CHAIN_WAVE_MIN="256", SMEM_CHAIN_REPLAY_CACHE="1"),
                                 dict(SMEM_CHAIN_HEAVY_MIN="0", SMEM_CHAIN_SORT_COUNT="0")],
                         ids=["all-wave", "all-lane", "lds-overflow", "tree-only", "tree-only-all-wave",
                              "serial-sort", "wave-cut-sort", "wave-cut-sort-hbm", "drop-pruned", "drop-hbm",
                              "one-launch", "rest-tier-hbm", "cluster-wave-all", "cluster-wave-256-cache",
                              "bitonic-close"])
def test_chain_paths_agree(gpu_device, monkeypatch, env):
    """The lane-per-read path, the wave-per-read paths (position clusters,
    and the chain tree they fall back to on equal chain keys), the wave
    path's HBM fallbacks (chain tree / filter records / drop-loop scratch
    beyond its LDS) and both drop loops (blocked, pruned) give the
    restatement's chains."""
    import smemgpu
    from smemgpu import synth
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = synth.make_genome(300_000, seed=81, repeat_frac=0.6, n_families=4, tandem_frac=0.01)
    idx, sa = smemgpu.Index.build_sa(g.codes, sa_intv=32)
    gpu = smemgpu.Gpu(idx, device=gpu_device)
    try:
        gpu.load_sa(sa)
        reads = synth.concat_reads([synth.make_reads(g.codes, 1500, 150, seed=82, sub_rate=0.01),
                                    synth.make_reads(g.codes, 300, (10, 250), seed=83)])
        b = gpu.batch(reads.n, reads.codes.size, int(reads.lens.max()))
        b.set_reads(reads.codes, reads.offs)
        b.run()
        b.sa(19, 10000)
        l_pac = idx.seq_len // 2
        for filt in (0, 1):
            b.chain(l_pac, filter=bool(filt), w=5, max_chain_gap=40)
            res = b.fetch()
            assert res.to_smch() == _oracle_chains(res, reads.n, l_pac, 19, 10000, filter=filt, w=5,
                                                   max_chain_gap=40)
        b.close()
    finally:
        gpu.close()


@pytest.mark.parametrize("env", [dict(), dict(SMEM_CHAIN_HEAVY_MIN="0"), dict(SMEM_CHAIN_HEAVY_MIN="0", SMEM_CHAIN_LDS="4096"),
                                 dict(SMEM_CHAIN_HEAVY_MIN="0", SMEM_CHAIN_REPLAY_CACHE="1"),
                                 dict(SMEM_CHAIN_HEAVY_MIN="0", SMEM_CHAIN_LDS="12288", SMEM_CHAIN_REPLAY_CACHE="1"),
                                 dict(SMEM_CHAIN_HEAVY_MIN="0", SMEM_CHAIN_WAVE_MIN="2")],
                         ids=["default", "all-wave", "all-wave-hbm-tree", "record-cache", "record-cache-shrinks",
                              "cluster-wave-all"])
def test_chain_equal_keys_replay(gpu_device, monkeypatch, env):
    """Reads X + Y + X whose two copies of X match one locus: test_and_merge
    rejects the far query offset, so two chains share a pos, and the
    position-cluster path hands the read to the kbtree replay (which of two
    equal keys the tree returns depends on its node layout).  Chains ==
    the restatement's, with and without the filter."""
    import smemgpu
    from smemgpu import synth
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = synth.make_genome(300_000, seed=91, repeat_frac=0.3, n_families=3, n_chrom=1)
    G = g.codes
    rng = np.random.default_rng(92)
    parts = []
    for r in range(600):
        p = int(rng.integers(0, G.size - 500))
        q = int(rng.integers(0, G.size - 500))
        x = G[p:p + int(rng.integers(25, 70))]
        parts.append(np.concatenate([x, G[q:q + int(rng.integers(101, 160))], x]).astype(np.uint8))
    base = synth.make_reads(G, 600, 150, seed=93, sub_rate=0.01)
    codes = np.concatenate(parts + [base.codes]).astype(np.uint8)
    lens = [x.size for x in parts] + list(np.diff(base.offs))
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    n = offs.size - 1
    idx, sa = smemgpu.Index.build_sa(G, sa_intv=32)
    gpu = smemgpu.Gpu(idx, device=gpu_device)
    try:
        gpu.load_sa(sa)
        b = gpu.batch(n, codes.size, int(np.max(lens)))
        b.set_reads(codes, offs)
        b.run()
        b.sa(19, 10000)
        l_pac = idx.seq_len // 2
        for filt in (0, 1):
            b.chain(l_pac, filter=bool(filt))
            res = b.fetch()
            assert res.to_smch() == _oracle_chains(res, n, l_pac, 19, 10000, filter=filt)
        b.close()
    finally:
        gpu.close()


@pytest.mark.parametrize("env", [dict(), dict(SMEM_CHAIN_STREAMS="1"), dict(SMEM_CHAIN_GIANT_MIN="256"),
                                 dict(SMEM_CHAIN_REPLAY_CACHE="1"), dict(SMEM_CHAIN_WAVE_MIN="256"),
                                 dict(SMEM_CHAIN_SORT_COUNT="0"), dict(SMEM_CHAIN_GIANT_ORDER="1"),
                                 dict(SMEM_CHAIN_STREAMS="1", SMEM_CHAIN_GIANT_MIN="256", SMEM_CHAIN_GIANT_ORDER="1"),
                                 dict(SMEM_CHAIN_GIANT_ORDER="2", SMEM_CHAIN_GIANT_WAVES="3")],
                         ids=["tiers", "one-launch", "more-giants", "record-cache", "cluster-wave-256", "bitonic-close",
                              "longest-first", "one-launch-longest-first", "shortest-first-3-waves"])
def test_chain_human_like_giants(gpu_device, monkeypatch, env):
    """A 4 Mbp genome with the human-like repeat profile and 8 % satellite /
    simple-sequence arrays: reads from the arrays carry thousands of seed
    occurrences (the giant LDS tier, > 2048), thousands of chains per read
    (rank-bitmap clusters, the kbtree replay, the two-pass drop loop with its
    kept list past the 64 register slots).  Chains == the restatement's, with
    and without the filter, in both heavy-read launch layouts, with the giants
    in listing order (the default), longest or shortest first, on a few waves."""
    import smemgpu
    from smemgpu import synth
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = synth.make_genome_human_like(4_000_000, seed=5, n_chrom=2, satellite_frac=0.08)
    idx, sa = smemgpu.Index.build_sa(g.codes, sa_intv=32)
    reads = synth.make_reads(g.codes, 4000, 150, seed=6, sub_rate=0.01)
    gpu = smemgpu.Gpu(idx, device=gpu_device)
    try:
        gpu.load_sa(sa)
        b = gpu.batch(reads.n, reads.codes.size, int(reads.lens.max()))
        b.set_reads(reads.codes, reads.offs)
        b.run()
        b.sa(19, 10000)
        l_pac = idx.seq_len // 2
        for filt in (0, 1):
            b.chain(l_pac, filter=bool(filt))
            res = b.fetch()
            n_occ = np.array([res.read_sa(i).size for i in range(reads.n)])
            n_chain = np.diff(res.chain_off)
            assert n_occ.max() > 2048 and (n_occ > 256).sum() >= 16
            assert n_chain.max() > (1000 if not filt else 64)
            assert res.to_smch() == _oracle_chains(res, reads.n, l_pac, 19, 10000, filter=filt)
        b.close()
    finally:
        gpu.close()

"""The streaming path (smem_gpu_seed_stream): bwa mem's chunk loop with
kt_for_batch-style workers (software/fastmap.c:213-228,
software/bwamem.c:1614-1640, software/kthread_batch.c:29-59) over host
buffers.  Bar: every chunk's lists, reassembled in chunk order, equal the
oracle's lists for the whole read set, bit for bit, whatever the chunk size,
worker count and completion order; pairs keep both mates in one chunk
(software/bwamem.c:1600-1609)."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def world(gpu_device):
    import smemgpu
    from smemgpu import synth
    g = synth.make_genome_human_like(1_500_000, seed=31)
    idx = smemgpu.Index.build(g.codes)
    gpu = smemgpu.Gpu(idx, device=gpu_device)
    ref = oracle.OracleIndex(words=idx.words, primary=idx.primary, L2=idx.L2)
    yield dict(codes=g.codes, gpu=gpu, ref=ref)
    gpu.close()
    ref.close()


def _joined(chunks, n_reads):
    from smemgpu.lib import Results
    iv = np.concatenate([c.intv for c in chunks]) if chunks else np.zeros((0, 4), np.uint64)
    cn = np.concatenate([c.call_n for c in chunks]) if chunks else np.zeros(0, np.uint32)
    io, co = [np.uint64(0)], [np.uint64(0)]
    for c in chunks:
        io.extend(list(c.intv_off[1:] + io[-1]))
        co.extend(list(c.call_off[1:] + co[-1]))
    r = Results(iv, np.array(io, dtype=np.uint64), cn, np.array(co, dtype=np.uint64))
    assert r.intv_off.size == n_reads + 1
    return r


@pytest.mark.parametrize("chunk,workers,packed", [(997, 3, False), (4096, 2, True), (50_000, 1, False), (1, 4, True),
                                                  (1500, 4, True)])
def test_stream_equals_oracle(world, chunk, workers, packed):
    import smemgpu
    from smemgpu import synth
    n = 6000 if chunk > 1 else 40
    reads = synth.make_reads(world["codes"], n, 150, seed=chunk, sub_rate=0.03, n_rate=0.002)
    want, _, _ = oracle.seed(world["ref"], reads.codes, reads.offs, threads=8)
    st, chunks = world["gpu"].seed_stream(reads.codes, reads.offs, smemgpu.Options(), chunk_reads=chunk,
                                          workers=workers, collect=True, packed=packed)
    assert st["n_reads"] == n and st["n_chunks"] == (n + chunk - 1) // chunk
    assert st["workers"] == min(workers, st["n_chunks"])
    assert _joined(chunks, n).to_smgo() == want
    assert st["n_intv"] == sum(int(c.intv_off[-1]) for c in chunks)
    assert st["d2h_bytes"] >= (16 if packed else 32) * st["n_intv"]


def test_stream_pairs(world):
    """Interleaved mates: odd chunk sizes are rounded down to even, so no pair
    is split; an odd read count is refused."""
    import smemgpu
    from smemgpu import synth
    reads = synth.make_pairs(world["codes"], 2500, 150, seed=7)
    want, _, _ = oracle.seed(world["ref"], reads.codes, reads.offs, threads=8)
    st, chunks = world["gpu"].seed_stream(reads.codes, reads.offs, smemgpu.Options(), chunk_reads=1001, workers=3,
                                          pairs=True, collect=True, packed=True)
    assert all((c.intv_off.size - 1) % 2 == 0 for c in chunks)
    assert st["n_chunks"] == (5000 + 999) // 1000
    assert _joined(chunks, 5000).to_smgo() == want
    odd = reads.subset(np.arange(4999))
    with pytest.raises(smemgpu.SmemError):
        world["gpu"].seed_stream(odd.codes, odd.offs, pairs=True)


def test_stream_options_and_edges(world):
    import smemgpu
    from smemgpu import synth
    reads = synth.concat_reads([synth.make_reads(world["codes"], 700, (1, 300), seed=3, n_rate=0.02),
                                synth.make_reads(world["codes"], 300, 250, seed=4, sub_rate=0.05)])
    for opt in (dict(min_seed_len=14, split_width=20), dict(start_width=2), dict(split_factor=1.0, split_width=500)):
        want, _, _ = oracle.seed(world["ref"], reads.codes, reads.offs, threads=8, **opt)
        _, chunks = world["gpu"].seed_stream(reads.codes, reads.offs, smemgpu.Options(**opt), chunk_reads=333,
                                             workers=3, collect=True)
        assert _joined(chunks, reads.n).to_smgo() == want
    empty = synth.make_reads(world["codes"], 0, 150, seed=1)
    st, chunks = world["gpu"].seed_stream(empty.codes, empty.offs, collect=True)
    assert st["n_reads"] == 0 and chunks == []


def test_stream_pool_reuse_and_release(world):
    """Batches kept from a 4-worker call serve a 2-worker call (the pool then
    shrinks to 2), SMEM_STREAM_RELEASE empties it, and the next call builds
    fresh batches: every result equals the oracle's."""
    import smemgpu
    from smemgpu import synth
    reads = synth.make_reads(world["codes"], 3000, 150, seed=11, sub_rate=0.03)
    want, _, _ = oracle.seed(world["ref"], reads.codes, reads.offs, threads=8)
    for workers, release in ((4, False), (2, False), (3, True), (2, False)):
        st, chunks = world["gpu"].seed_stream(reads.codes, reads.offs, smemgpu.Options(), chunk_reads=500,
                                              workers=workers, collect=True, packed=True, release=release)
        assert st["workers"] == workers
        assert _joined(chunks, reads.n).to_smgo() == want


def test_pintv_roundtrip_limits(world):
    """The 16-B wire entry carries 34-bit coordinates and 13-bit query
    positions; reads past 8191 bp are refused in packed mode."""
    import smemgpu
    from smemgpu import synth
    from smemgpu.lib import unpack_pintv
    x = np.array([[(1 << 34) - 1, 5, (1 << 33) + 7, (8191 << 32) | 8191]], dtype=np.uint64)
    w = (x[:, 0] >> 32) | (x[:, 1] >> 32) << 2 | (x[:, 2] >> 32) << 4 | (x[:, 3] >> 32) << 6 | (x[:, 3] & 8191) << 19
    p = np.stack([x[:, 0] & 0xffffffff, x[:, 1] & 0xffffffff, x[:, 2] & 0xffffffff, w], axis=1).astype(np.uint32)
    assert np.array_equal(unpack_pintv(p), x)
    long = synth.make_reads(world["codes"], 2, 9000, seed=1)
    with pytest.raises(smemgpu.SmemError):
        world["gpu"].seed_stream(long.codes, long.offs, packed=True)

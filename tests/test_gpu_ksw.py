"""GPU parity of the SW extension kernel, through the
C ABI: smem_ksw_extend == ksw_extend2 (software/ksw.c:379-476) on every task,
all six outputs (score, qle, tle, gtle, gscore, max_off), bit-exact.

Checked against the compiled reference's own results (tests/golden/ksw.*,
5000 problems shaped like mem_chain2aln's left/right extensions) and against
the restatement (oracle/ksw_oracle.c, pinned to those) on fresh problems under
other scoring, band widths, z-drop settings and query lengths up to the limit.
"""
import numpy as np
import pytest

from oracle import oracle
from tests import golden_data

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["wave", "wave_unsorted", "g16", "lane"], autouse=True)
def ksw_kernel(request, monkeypatch):
    """Every test on each kernel: one problem per wave (the problems in
    query-length order, the default, and in the caller's order:
    SMEM_KSW_SORT=0), four per wave on 16-lane groups (SMEM_KSW_G16,
    kswd::extend_group16), and one per lane (SMEM_KSW_LANE, kswl::extend_lane,
    with its fallbacks to one per wave)."""
    if request.param == "wave_unsorted":
        monkeypatch.setenv("SMEM_KSW_SORT", "0")
    if request.param == "g16":
        monkeypatch.setenv("SMEM_KSW_G16", "1")
    if request.param == "lane":
        monkeypatch.setenv("SMEM_KSW_LANE", "1")
    return request.param


@pytest.fixture(scope="module")
def gpu(gpu_device):
    import smemgpu
    from smemgpu import synth
    g = synth.make_genome(20_000, seed=141, n_chrom=1)
    idx = smemgpu.Index.build(g.codes)
    h = smemgpu.Gpu(idx, device=gpu_device)
    yield h
    h.close()


def test_ksw_golden_fixture(gpu):
    from smemgpu import synth
    b = synth.read_smkt(golden_data.gz("ksw.smkt.gz"))
    want = synth.read_smkr(golden_data.gz("ksw.smkr.gz"))
    got, _ = gpu.ksw_extend(b)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("scoring", ["bwa", "a2b3", "asym"])
def test_ksw_vs_oracle(gpu, scoring):
    from smemgpu import synth
    g = synth.make_genome(400_000, seed=142, n_chrom=1)
    b = synth.make_ksw_tasks(g.codes, 6000, seed=143 + len(scoring))
    if scoring == "a2b3":
        b.mat = synth.bwa_scmat(2, 3)
    elif scoring == "asym":
        b.mat = synth.bwa_scmat(1, 4)
        b.o_del, b.e_del, b.o_ins, b.e_ins = 5, 3, 8, 1
    got, ms = gpu.ksw_extend(b)
    want = oracle.ksw(b)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:5], b.tasks[bad[:5]], got[bad[:5]], want[bad[:5]])
    assert ms > 0


def test_ksw_edges(gpu):
    """qlen 1 and 255 (the column limit), empty targets, h0 = 0, z-drop off,
    bands of 1, all-N queries, scores past 16 bits (h0 near 2^16: the lane
    kernel hands those to one wave each), query lengths at the lane tiers'
    edges (32, 33, 64, 65, 128, 129)."""
    from smemgpu import synth
    rng = np.random.default_rng(150)
    tasks, qs, ts = [], [], []
    qo = to = 0
    for qlen, tlen, w, zd, h0 in [(1, 0, 100, 100, 10), (1, 1, 100, 100, 0), (255, 300, 100, 100, 40),
                                  (255, 255, 1, 0, 200), (200, 0, 100, 100, 30), (64, 64, 5, 100, 19),
                                  (65, 130, 200, 100, 100), (128, 90, 100, 0, 0), (191, 192, 50, 3, 60),
                                  (100, 120, 100, 100, 65500), (30, 40, 100, 100, 65400), (32, 40, 10, 100, 30),
                                  (33, 50, 100, 100, 30), (129, 140, 100, 100, 50), (8, 300, 100, 0, 20)]:
        for rep in range(3):
            q = rng.integers(0, 4, size=qlen).astype(np.uint8)
            t = np.concatenate([q[:min(qlen, tlen)], rng.integers(0, 4, size=max(0, tlen - qlen))]).astype(np.uint8)
            if rep == 1 and tlen:
                hit = rng.random(t.size) < 0.1
                t[hit] = (t[hit] + 1) & 3
            if rep == 2:
                q[:] = 4
            tasks.append((qo, to, qlen, t.size, w, 5, zd, h0))
            qs.append(q)
            ts.append(t)
            qo += q.size
            to += t.size
    b = synth.KswBatch(np.array(tasks, dtype=synth.KSW_TASK), np.concatenate(qs), np.concatenate(ts),
                       synth.bwa_scmat())
    got, _ = gpu.ksw_extend(b)
    assert np.array_equal(got, oracle.ksw(b))


def test_ksw_rejects(gpu):
    import smemgpu
    from smemgpu import synth
    b = synth.KswBatch(np.array([(0, 0, 256, 10, 100, 5, 100, 10)], dtype=synth.KSW_TASK),
                       np.zeros(256, np.uint8), np.zeros(10, np.uint8), synth.bwa_scmat())
    with pytest.raises(smemgpu.SmemError):
        gpu.ksw_extend(b)
    b.tasks["qlen"] = 0
    with pytest.raises(smemgpu.SmemError):
        gpu.ksw_extend(b)
    b.tasks["qlen"] = 5
    b.tasks["t_off"] = 8  # past the target pool
    with pytest.raises(smemgpu.SmemError):
        gpu.ksw_extend(b)
    e = synth.KswBatch(np.zeros(0, dtype=synth.KSW_TASK), np.zeros(0, np.uint8), np.zeros(0, np.uint8),
                       synth.bwa_scmat())
    got, _ = gpu.ksw_extend(e)
    assert got.size == 0

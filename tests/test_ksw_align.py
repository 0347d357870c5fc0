"""ksw_align2 (software/ksw.c:342-364, ksw_u8 / ksw_i16 :110-333): the local SW
of mem_chain2aln_short (software/bwamem.c:805-852).

Golden: tests/golden/kswa_a<1|2>.smat/.smar, the compiled reference's own
ksw_align2 on 3000 problems each, shaped like the short path (query span of
the seeds + 50 each side, < 200 bp, against the reference span + 50), under
mem_opt_init's scoring (a = 1: every problem byte-scored) and -A 2 scaling
(a = 2: queries from 125 bp on take the 16-bit branch).  Bar: all seven
kswr_t fields bit-exact, for the restatement (CPU) and the GPU's wave routine
(the one the alignment kernel runs, through smem_ksw_align2)."""
import gzip
import os

import numpy as np
import pytest

from oracle import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
SETS = ["kswa_a1", "kswa_a2"]


def _load(name):
    from smemgpu import synth
    with gzip.open(os.path.join(HERE, "golden", name + ".smat.gz"), "rb") as fh:
        kb = synth.read_smat(fh.read())
    with gzip.open(os.path.join(HERE, "golden", name + ".smar.gz"), "rb") as fh:
        want = synth.read_smar(fh.read())
    return kb, want


def _same(got, want):
    for f in want.dtype.names:
        bad = np.nonzero(got[f] != want[f])[0]
        assert bad.size == 0, f"{f}: {bad.size} differ, first {bad[:5]}"


@pytest.mark.parametrize("name", SETS)
def test_kswa_fixture_shape(name):
    kb, want = _load(name)
    assert kb.tasks.size == want.size == 3000
    byte = (kb.tasks["xtra"] & 0x10000) != 0
    if name == "kswa_a2":
        assert (~byte).sum() > 500          # the 16-bit branch runs
    assert (want["tb"] >= 0).sum() > 1000   # the start pass runs
    assert (want["score2"] > 0).sum() > 100  # suboptimal hits
    assert (want["te2"] >= 0).sum() > 100


@pytest.mark.parametrize("name", SETS)
def test_kswa_oracle_vs_reference(name):
    kb, want = _load(name)
    _same(oracle.ksw_align2(kb), want)


@pytest.mark.gpu
@pytest.mark.parametrize("name", SETS)
def test_kswa_gpu_vs_reference(gpu_device, name):
    import smemgpu
    kb, want = _load(name)
    idx = smemgpu.Index.build(np.random.default_rng(1).integers(0, 4, 5000).astype(np.uint8))
    gpu = smemgpu.Gpu(idx, device=gpu_device)
    try:
        got, ms = gpu.ksw_align2(kb)
    finally:
        gpu.close()
    _same(got, want)

"""End-to-end parity of the reference-side binding (integration/): the
reference's own `bwa` CLI with the maintainer's patch applied
(integration/patches: main.c, bwa.c, fastmap.c, bwamem.c) and linked to
libsmemgpu.so, built by integration/Makefile into oracle/_ref/bwa-gpu.

Golden: tests/golden/sam/*.sam.gz, the unpatched reference pipeline's SAM
(`bwa mem -t 1 -b 1`, tests/golden/make_golden_sam.py).  Bar: byte-identical
SAM apart from the @PG line -- north_star: "the `bwa mem` CLI and downstream
chaining/SAM path are unchanged".

* CPU (always): without a usable device the patched mem_chain_batched takes the
  reject -> CPU path (mem_chain); SAM must still be identical.
* GPU (-m gpu): seeding, bwt_sa and chaining of every kt_for_batch worker batch
  run on the MI355X (smem_gpu_collect -> smem_batch_sa -> smem_batch_chain),
  SW extension / pairing / SAM on the CPU, unchanged.
"""
import gzip
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BWA = os.path.join(ROOT, "oracle", "_ref", "bwa-gpu")
GOLD = os.path.join(ROOT, "tests", "golden")
CASES = [("g1", "se"), ("g1", "pe"), ("g2", "se"), ("g2", "pe")]


def _need_bwa():
    if not os.path.exists(BWA):
        pytest.skip("oracle/_ref/bwa-gpu not built (make -C integration needs /root/reference)")


@pytest.fixture(scope="module")
def indexed(tmp_path_factory, built):
    """g1 / g2 indexed by the reference's own `bwa index -a is` (inside bwa-gpu)."""
    _need_bwa()
    d = tmp_path_factory.mktemp("bwa")
    out = {}
    for g in ("g1", "g2"):
        fa = d / f"{g}.fa"
        with gzip.open(os.path.join(GOLD, f"{g}.fa.gz"), "rb") as src, open(fa, "wb") as dst:
            shutil.copyfileobj(src, dst)
        subprocess.run([BWA, "index", "-a", "is", str(fa)], check=True, capture_output=True, cwd=d)
        out[g] = str(fa)
    return out


def _golden(g, kind) -> list:
    with gzip.open(os.path.join(GOLD, "sam", f"{g}_{kind}.sam.gz"), "rt") as fh:
        return [l for l in fh.read().split("\n") if l and not l.startswith("@PG")]


def _run(fa, g, kind, threads, batch, env=None):
    args = [BWA, "mem", "-t", str(threads), "-b", str(batch)] + (["-p"] if kind == "pe" else []) + \
           [fa, os.path.join(GOLD, "sam", f"{g}_{kind}.fq.gz")]
    p = subprocess.run(args, capture_output=True, text=True, env=dict(os.environ, **(env or {})), timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    return [l for l in p.stdout.split("\n") if l and not l.startswith("@PG")], p.stderr


@pytest.mark.parametrize("g,kind", CASES)
def test_cpu_fallback_sam_identical(indexed, g, kind):
    """No device (or a refused one): the patched build seeds on the CPU and
    the SAM equals the reference's."""
    got, err = _run(indexed[g], g, kind, 3, 64, env={"SMEM_GPU_DEVICE": "63"})
    assert "seeding on the CPU" in err
    assert got == _golden(g, kind)


@pytest.mark.gpu
@pytest.mark.parametrize("g,kind", CASES)
@pytest.mark.parametrize("threads,batch", [(4, 4096), (3, 37)])
def test_gpu_sam_identical(indexed, gpu_device, g, kind, threads, batch):
    """Seeding + bwt_sa + mem_chain on the MI355X behind mem_chain_batched:
    SAM byte-identical to the reference's `bwa mem -t 1 -b 1`."""
    got, err = _run(indexed[g], g, kind, threads, batch)
    assert "seeding on the CPU" not in err, err[-2000:]
    want = _golden(g, kind)
    assert len(got) == len(want)
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    assert not bad, f"{len(bad)} SAM lines differ, first: {got[bad[0]][:200]} vs {want[bad[0]][:200]}"

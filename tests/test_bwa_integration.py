"""End-to-end parity of the reference-side binding (integration/): the
reference's own `bwa` CLI with the maintainer's patch applied
(integration/patches: main.c, bwa.c, fastmap.c, bwamem.c, bwtindex.c) and linked to
libsmemgpu.so, built by integration/Makefile into oracle/_ref/bwa-gpu.

Golden: tests/golden/sam/*.sam.gz, the unpatched reference pipeline's SAM
(`bwa mem -t 1 -b 1`, tests/golden/make_golden_sam.py).  Bar: byte-identical
SAM apart from the @PG line -- north_star: "the `bwa mem` CLI and downstream
chaining/SAM path are unchanged".

* CPU (always): without a usable device the patched mem_align1_core_batched
  takes the reject -> CPU path (mem_chain); SAM must still be identical.
* GPU (-m gpu): the seeding loop, bwt_sa, mem_chain + mem_chain_flt and
  mem_chain2aln_short / mem_chain2aln of every kt_for_batch worker batch run on
  the MI355X (smem_gpu_collect_ex -> smem_batch_sa -> smem_batch_chain(filter)
  -> smem_batch_chain2aln -> regions only), mem_sort_and_dedup / pairing / SAM
  on the CPU, unchanged; also SMEM_GPU_STAGES=1 (chains back, filter and
  extension on the CPU), two device contexts (SMEM_GPU_DEVICES=0,0: worker tid
  on context tid % 2), and reads > 1024 bp (chains -> regions refused, the
  GPU-filtered chains extended on the CPU), the last against the compiled
  reference run on the same reads here.
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
    if os.path.exists(BWA + ".FAILED"):  # written by __graft_entry__.build() when make -C integration failed
        pytest.fail("oracle/_ref/bwa-gpu failed to build: " + open(BWA + ".FAILED").read().strip())
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
        # the reference's CPU steps (the GPU build of `bwa index` is tested
        # against them below)
        subprocess.run([BWA, "index", "-a", "is", str(fa)], check=True, capture_output=True, cwd=d,
                       env=dict(os.environ, SMEM_GPU_INDEX="0"))
        out[g] = str(fa)
    return out


INDEX_FILES = (".bwt", ".sa", ".pac", ".ann", ".amb")


def _index_files(tmp, g, name, algo, env):
    """`bwa-gpu index [-a algo] -p <name>` of golden genome g in tmp -> (stderr, {suffix: bytes})."""
    fa = tmp / f"{g}.fa"
    if not fa.exists():
        with gzip.open(os.path.join(GOLD, f"{g}.fa.gz"), "rb") as src, open(fa, "wb") as dst:
            shutil.copyfileobj(src, dst)
    args = [BWA, "index"] + (["-a", algo] if algo else []) + ["-p", str(tmp / name), str(fa)]
    p = subprocess.run(args, capture_output=True, text=True, cwd=tmp, env=dict(os.environ, **env), timeout=900)
    assert p.returncode == 0, p.stderr[-2000:]
    return p.stderr, {x: open(tmp / (name + x), "rb").read() for x in INDEX_FILES}


def test_index_without_gpu_runs_the_reference_steps(tmp_path, built):
    """`bwa index` with no usable device (device 63: refused): the reference's
    CPU steps, announced, and the same files as with SMEM_GPU_INDEX=0."""
    _need_bwa()
    err, files = _index_files(tmp_path, "g1", "cpu", "is", {"SMEM_GPU_DEVICES": "63"})
    assert "the CPU builds the BWT and the SA" in err and "Update BWT" in err, err[-2000:]
    err0, ref = _index_files(tmp_path, "g1", "ref", "is", {"SMEM_GPU_INDEX": "0"})
    assert "Construct BWT and SA on GPU" not in err0
    assert files == ref


@pytest.mark.parametrize("g", ["g1", "g2"])
def test_index_host_builder_glue(tmp_path, built, g):
    """The patched `bwa index` glue (the forward strand read back from the
    .pac, the .bwt / .sa written in the reference's formats) run with the
    library's host builder (SMEM_GPU_INDEX=host): five files identical to the
    reference's CPU steps'."""
    _need_bwa()
    err, got = _index_files(tmp_path, g, "host", "is", {"SMEM_GPU_INDEX": "host"})
    assert "host builder" in err and "Update BWT" not in err, err[-2000:]
    _, want = _index_files(tmp_path, g, "cpu", "is", {"SMEM_GPU_INDEX": "0"})
    for x in INDEX_FILES:
        assert got[x] == want[x], x


@pytest.mark.gpu
@pytest.mark.parametrize("g", ["g1", "g2"])
@pytest.mark.parametrize("algo", ["is", None])
def test_gpu_index_files_identical(tmp_path, gpu_device, built, g, algo):
    """`bwa index` on the MI355X (smem_bwt_build_gpu_sa in place of the BWT
    construction, bwt_bwtupdate_core and bwt_cal_sa): all five index files
    byte-identical to the reference's CPU steps."""
    _need_bwa()
    err, got = _index_files(tmp_path, g, "gpu", algo, {})
    assert "Construct BWT and SA on GPU" in err and "Update BWT" not in err, err[-2000:]
    _, want = _index_files(tmp_path, g, "cpu", algo, {"SMEM_GPU_INDEX": "0"})
    for x in INDEX_FILES:
        assert got[x] == want[x], x


def _golden(g, kind) -> list:
    with gzip.open(os.path.join(GOLD, "sam", f"{g}_{kind}.sam.gz"), "rt") as fh:
        return [l for l in fh.read().split("\n") if l and not l.startswith("@PG")]


def _run(fa, g, kind, threads, batch, env=None):
    """batch None: no -b (the binding's batch plan)."""
    args = [BWA, "mem", "-t", str(threads)] + ([] if batch is None else ["-b", str(batch)]) + \
           (["-p"] if kind == "pe" else []) + [fa, os.path.join(GOLD, "sam", f"{g}_{kind}.fq.gz")]
    # SMEM_GPU_CRASH_TRACE: a host crash prints its backtrace (the library's handler); the whole
    # stderr of a failed run is kept under gpurun_out/ (merged back from a GPU box)
    p = subprocess.run(args, capture_output=True, text=True,
                       env=dict(os.environ, SMEM_GPU_CRASH_TRACE="1", **(env or {})), timeout=600)
    if p.returncode != 0:
        d = os.path.join(ROOT, "gpurun_out", "bwa_fail")
        os.makedirs(d, exist_ok=True)
        tag = f"{g}_{kind}_t{threads}_b{batch}_" + "_".join(f"{k}={v}" for k, v in (env or {}).items()).replace(",", ".")
        with open(os.path.join(d, tag[:120] + ".err"), "w") as fh:
            fh.write(" ".join(args) + "\n" + p.stderr)
    crash = p.stderr.find("[smem crash]")
    assert p.returncode == 0, (p.stderr[crash:crash + 3000] if crash >= 0 else p.stderr[-2000:])
    return [l for l in p.stdout.split("\n") if l and not l.startswith("@PG")], p.stderr


@pytest.mark.parametrize("g,kind", CASES)
def test_cpu_fallback_sam_identical(indexed, g, kind):
    """No device (or a refused one): the patched build seeds on the CPU and
    the SAM equals the reference's."""
    got, err = _run(indexed[g], g, kind, 3, 64, env={"SMEM_GPU_DEVICES": "63"})
    assert "seeding on the CPU" in err
    assert got == _golden(g, kind)


def _same(got, want):
    assert len(got) == len(want)
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    if bad:
        def fields(i):  # the fields that differ (SEQ / QUAL cut short)
            a, b = got[i].split("\t"), want[i].split("\t")
            return [(k, x[:60], y[:60]) for k, (x, y) in enumerate(zip(a, b)) if x != y] + \
                [("n_fields", len(a), len(b))] * (len(a) != len(b))
        detail = "; ".join(f"{got[i].split(chr(9))[0]}: {fields(i)}" for i in bad[:6])
        raise AssertionError(f"{len(bad)} SAM lines differ (lines {bad[:12]}): {detail}")


GPU_MODES = {
    "regions": {},                             # default: seeding -> regions on the GPU
    "chains": {"SMEM_GPU_STAGES": "1"},        # seeding -> chains on the GPU (round-2 binding)
    "two_ctx": {"SMEM_GPU_DEVICES": "0,0"},    # two device contexts, workers dealt tid % 2
    "sa_raw": {"SMEM_GPU_SA_RAW": "1"},        # SA lookups to the uploaded samples (as before the densification ends)
}


@pytest.mark.gpu
@pytest.mark.parametrize("g,kind", CASES)
@pytest.mark.parametrize("threads,batch", [(4, 4096), (3, 37)])
@pytest.mark.parametrize("mode", sorted(GPU_MODES))
def test_gpu_sam_identical(indexed, gpu_device, g, kind, threads, batch, mode):
    """Seeding -> regions (or -> chains) on the MI355X behind
    mem_align1_core_batched: SAM byte-identical to the reference's
    `bwa mem -t 1 -b 1`."""
    got, err = _run(indexed[g], g, kind, threads, batch, env=GPU_MODES[mode])
    assert "seeding on the CPU" not in err and "refused" not in err, err[-2000:]
    if mode == "two_ctx":
        assert "2 GPU context(s)" in err, err[-2000:]
    _same(got, _golden(g, kind))


@pytest.mark.gpu
@pytest.mark.parametrize("g,kind", CASES)
@pytest.mark.parametrize("batch", [None, 4096, 37])
def test_gpu_sam_identical_eight_contexts(indexed, gpu_device, g, kind, batch):
    """The N = 8 fan-out on one GPU: SMEM_GPU_DEVICES=0,0,0,0,0,0,0,0 opens
    eight device contexts (index, .sa, .pac and worker slots each), `-t 16`
    deals worker tid to context tid % 8 / slot tid / 8 (software/fastmap.c:
    204-210's per-worker buffers, one manager per device).  Without -b the
    batch plan deals each context its share of the chunk in batches whose
    admitted ones hold a seeding grid together -- a share under one grid
    (these small inputs) is one batch: 8 batches, 8 workers.  SAM
    byte-identical to the reference's.  SMEM_GPU_SA_CHECK: the eight handles'
    densified SAs are one array (round 6: with the densification's scratch
    from the process-wide memory pool, one handle's came out different in
    ~15 % of runs, and bwa mem crashed or printed wrong records)."""
    got, err = _run(indexed[g], g, kind, 16, batch,
                    env={"SMEM_GPU_DEVICES": ",".join(["0"] * 8), "SMEM_GPU_TIMES": "1", "SMEM_GPU_SA_CHECK": "1"})
    assert "seeding on the CPU" not in err and "refused" not in err, err[-2000:]
    assert "8 GPU context(s)" in err, err[-2000:]
    import re
    checks = re.findall(r"\[M::sa_check\] handle \S+ device \d+: (\d+) of \d+ stored samples differ from the dense SA "
                        r"\(dense hash ([0-9a-f]+)\)", err)
    assert len(checks) == 8 and all(c[0] == "0" for c in checks) and len({c[1] for c in checks}) == 1, checks
    _same(got, _golden(g, kind))
    if batch is None:
        sizes = [int(m) for m in re.findall(r"\[M::mem_batch_gpu\] (\d+) reads through the GPU stages", err)]
        done = [int(m) for m in re.findall(r"\[M::mem_process_seqs\] Processed (\d+) reads", err)]
        assert len(sizes) == 8 * len(done) and sum(sizes) == sum(done), (sizes, done)


@pytest.mark.gpu
def test_gpu_long_reads_sam_identical(indexed, gpu_device, tmp_path):
    """Reads of 30-2000 bp (every batch holds some > 1024 bp, which
    smem_batch_chain2aln refuses): the GPU-filtered chains are extended on the
    CPU; SAM equals the compiled reference's `-b 1` run on the same reads
    (oracle/_ref/ref_harness mem, built from the reference sources)."""
    import numpy as np
    from smemgpu import synth
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(ref):
        pytest.fail("oracle/_ref/ref_harness missing (built by __graft_entry__.build() where /root/reference exists)")
    fa = indexed["g1"]
    seq = []
    with open(fa, "rb") as fh:
        for line in fh:
            if not line.startswith(b">"):
                seq.append(line.strip())
    codes = synth.NT4[np.frombuffer(b"".join(seq), dtype=np.uint8)]
    r = synth.make_reads(codes, 600, (30, 2000), seed=31, sub_rate=0.02, n_rate=0.002, random_frac=0.05)
    fq = tmp_path / "long.fq"
    acgtn = np.frombuffer(b"ACGTN", dtype=np.uint8)
    with open(fq, "wb") as fh:
        for i in range(r.n):
            s = acgtn[np.minimum(r.read(i), 4)].tobytes()
            fh.write(b"@l%d\n" % i + s + b"\n+\n" + b"I" * len(s) + b"\n")
    p = subprocess.run([ref, "mem", fa, str(fq), "4", "1", "0"], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    want = [l for l in p.stdout.split("\n") if l and not l.startswith("@PG")]
    args = [BWA, "mem", "-t", "3", "-b", "128", fa, str(fq)]
    q = subprocess.run(args, capture_output=True, text=True, timeout=600)
    assert q.returncode == 0, q.stderr[-2000:]
    assert "seeding on the CPU" not in q.stderr, q.stderr[-2000:]
    _same([l for l in q.stdout.split("\n") if l and not l.startswith("@PG")], want)


def test_bwa_prefix_from_smem_index_matches_bwa_index(tmp_path, built):
    """bench.py's e2e leg builds the human-size bwa index prefix from this
    repo's own .bwt / .sa plus synth.write_bwa_bns (.pac / .ann / .amb): on a
    small genome cut the same way, all five files equal the reference's own
    `bwa index -a is` output byte for byte."""
    _need_bwa()
    import smemgpu
    from smemgpu import synth
    g = synth.make_genome(250_000, seed=77)
    fa = tmp_path / "c.fa"
    synth.write_fasta_contigs(str(fa), g.codes, n_contigs=5)
    subprocess.run([BWA, "index", "-a", "is", str(fa)], check=True, capture_output=True)
    mine = str(tmp_path / "m")
    idx, sa = smemgpu.Index.build_sa(g.codes, sa_intv=32)
    idx.write(mine + ".bwt")
    sa.write(mine + ".sa")
    synth.write_bwa_bns(mine, g.codes, n_contigs=5)
    for ext in (".bwt", ".sa", ".pac", ".ann", ".amb"):
        assert open(mine + ext, "rb").read() == open(str(fa) + ext, "rb").read(), ext


@pytest.fixture(scope="module")
def two_chunks(indexed, tmp_path_factory):
    """75k x 150 bp reads of g1 (11.25 M bases: two `bwa mem -t 1` chunks of
    10 M bases) and the compiled reference's SAM of them (ref_harness mem,
    the reference's sequential chunk loop)."""
    import numpy as np
    from smemgpu import synth
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(ref):
        pytest.fail("oracle/_ref/ref_harness missing (built by __graft_entry__.build() where /root/reference exists)")
    fa = indexed["g1"]
    seq = []
    with open(fa, "rb") as fh:
        for line in fh:
            if not line.startswith(b">"):
                seq.append(line.strip())
    codes = synth.NT4[np.frombuffer(b"".join(seq), dtype=np.uint8)]
    r = synth.make_reads(codes, 75_000, 150, seed=77, sub_rate=0.02, n_rate=0.001, random_frac=0.02)
    fq = tmp_path_factory.mktemp("chunks") / "r.fq"
    acgtn = np.frombuffer(b"ACGTN", dtype=np.uint8)
    with open(fq, "wb") as fh:
        for i in range(r.n):
            s = acgtn[np.minimum(r.read(i), 4)].tobytes()
            fh.write(b"@c%d\n" % i + s + b"\n+\n" + b"I" * len(s) + b"\n")
    p = subprocess.run([ref, "mem", fa, str(fq), "1", "1", "0"], capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stderr[-2000:]
    return fa, str(fq), [l for l in p.stdout.split("\n") if l and not l.startswith("@PG")]


def _run_chunks(fa, fq, env):
    q = subprocess.run([BWA, "mem", "-t", "1", fa, fq], capture_output=True, text=True, timeout=900,
                       env=dict(os.environ, **env))
    assert q.returncode == 0, q.stderr[-2000:]
    assert q.stderr.count("[M::main_mem] read ") == 2, q.stderr[-2000:]
    return [l for l in q.stdout.split("\n") if l and not l.startswith("@PG")], q.stderr


def test_pipelined_chunks_sam_identical(two_chunks):
    """The patched main_mem's chunk pipeline (a reader thread parsing chunk
    k+1, a writer printing chunk k-1 while chunk k is processed) on the CPU
    path: SAM equal to the reference's sequential loop over two chunks."""
    fa, fq, want = two_chunks
    got, _ = _run_chunks(fa, fq, {"SMEM_GPU_DEVICES": "63"})
    _same(got, want)


@pytest.mark.gpu
def test_gpu_pipelined_chunks_sam_identical(two_chunks, gpu_device):
    """The same two chunks with the GPU stages (and the SE SAM beside them)
    under the chunk pipeline, and with SMEM_GPU_PIPELINE=0: both equal the
    reference's SAM."""
    fa, fq, want = two_chunks
    for env in ({}, {"SMEM_GPU_PIPELINE": "0"}):
        got, err = _run_chunks(fa, fq, env)
        assert "seeding on the CPU" not in err and "refused" not in err, err[-2000:]
        _same(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("g", ["g1", "g2"])
def test_gpu_pe_given_insert_sam_identical(indexed, gpu_device, g):
    """`bwa mem -p -I 500,50`: with the insert size given, the PE SAM of each
    pair is computed as soon as both mates' regions are back (no mem_pestat
    over the chunk); SAM equal to the same binary's reference CPU path and to
    its two-pass GPU run (SMEM_GPU_OVERLAP=0)."""
    _need_bwa()
    args = [BWA, "mem", "-t", "4", "-b", "256", "-p", "-I", "500,50", indexed[g],
            os.path.join(GOLD, "sam", f"{g}_pe.fq.gz")]

    def run(env):
        p = subprocess.run(args, capture_output=True, text=True, env=dict(os.environ, **env), timeout=600)
        assert p.returncode == 0, p.stderr[-2000:]
        return [l for l in p.stdout.split("\n") if l and not l.startswith("@PG")], p.stderr

    want, err = run({"SMEM_GPU_DEVICES": "63"})
    assert "seeding on the CPU" in err
    for env in ({}, {"SMEM_GPU_OVERLAP": "0"}):
        got, err = run(env)
        assert "seeding on the CPU" not in err and "refused" not in err, err[-2000:]
        _same(got, want)

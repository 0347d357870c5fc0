"""Deterministic synthetic genomes and reads for the SMEM seeding path.

There is no network and no human_g1k_v37 / E. coli index in this image, so
every benchmark and parity case runs on seeded synthetic data of the shapes
SURVEY.md §8(d) names (C1..C5): a random genome with diverged repeat families
and exact/tandem repeats, reads sampled from both strands with substitutions
and 0.1% ambiguous bases.

All randomness flows from numpy's PCG64 with an explicit seed, so the same
call always yields byte-identical output.

The file formats (SMRD reads, SMGO SMEM streams) are documented in
include/smem_formats.h.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

import numpy as np

NT4 = np.full(256, 4, dtype=np.uint8)  # software/bntseq.c:44 (nst_nt4_table)
for _ch, _v in zip(b"ACGTacgt", [0, 1, 2, 3, 0, 1, 2, 3]):
    NT4[_ch] = _v
NT4[ord("-")] = 5
ACGT = np.frombuffer(b"ACGTN", dtype=np.uint8)


@dataclass
class Genome:
    codes: np.ndarray        # uint8 0..3, all chromosomes concatenated
    chrom_names: list
    chrom_starts: np.ndarray  # int64 offsets into codes, len = n_chrom + 1


def _mutate(seq: np.ndarray, rate: float, rng: np.random.Generator) -> np.ndarray:
    out = seq.copy()
    if rate <= 0 or out.size == 0:
        return out
    hit = rng.random(out.size) < rate
    out[hit] = (out[hit] + rng.integers(1, 4, size=int(hit.sum()), dtype=np.uint8)) & 3
    return out


def make_genome(n_bp: int, seed: int = 1, n_chrom: int = 4, repeat_frac: float = 0.02,
                n_families: int = 200, exact_frac: float = 0.002, tandem_frac: float = 0.001) -> Genome:
    """Random genome with structure that exercises the SMEM path.

    - repeat_frac of the genome is overwritten by copies of n_families random
      families (300..3000 bp), each copy diverged by 0..15% substitutions and
      inserted on a random strand (multi-occurrence intervals, re-seeding);
    - exact_frac is covered by exact duplicated segments (long identical
      matches, x2 >= 2);
    - tandem_frac is covered by short-period tandem repeats / homopolymers
      (large intervals, max_occ filtering downstream).
    """
    rng = np.random.default_rng(seed)
    g = rng.integers(0, 4, size=n_bp, dtype=np.uint8)
    if n_bp >= 5000 and repeat_frac > 0:
        fam = [rng.integers(0, 4, size=int(rng.integers(300, 3001)), dtype=np.uint8) for _ in range(n_families)]
        budget = int(n_bp * repeat_frac)
        while budget > 0:
            f = fam[int(rng.integers(0, n_families))]
            div = float(rng.random() * 0.15)
            c = _mutate(f, div, rng)
            if rng.random() < 0.5:
                c = (3 - c)[::-1]
            if c.size >= n_bp:
                break
            p = int(rng.integers(0, n_bp - c.size))
            g[p:p + c.size] = c
            budget -= c.size
    if n_bp >= 20000 and exact_frac > 0:
        budget = int(n_bp * exact_frac)
        while budget > 0:
            ln = int(rng.integers(200, 2001))
            src = int(rng.integers(0, n_bp - ln))
            dst = int(rng.integers(0, n_bp - ln))
            seg = g[src:src + ln].copy()
            if rng.random() < 0.5:
                seg = (3 - seg)[::-1]
            g[dst:dst + ln] = seg
            budget -= ln
    if n_bp >= 20000 and tandem_frac > 0:
        budget = int(n_bp * tandem_frac)
        while budget > 0:
            period = int(rng.integers(1, 7))
            unit = rng.integers(0, 4, size=period, dtype=np.uint8)
            ln = int(rng.integers(20, 400))
            seg = np.resize(unit, ln)
            dst = int(rng.integers(0, n_bp - ln))
            g[dst:dst + ln] = seg
            budget -= ln
    n_chrom = max(1, min(n_chrom, n_bp // 1000 if n_bp >= 1000 else 1))
    cuts = np.sort(rng.choice(np.arange(1, n_bp), size=n_chrom - 1, replace=False)) if n_chrom > 1 else np.array([], dtype=np.int64)
    starts = np.concatenate([[0], cuts, [n_bp]]).astype(np.int64)
    names = [f"chr{i + 1}" for i in range(n_chrom)]
    return Genome(g, names, starts)


# Repeat profile shaped like human_g1k_v37's (RepeatMasker classes, roughly):
# (name, genome fraction, family length range, n families, divergence range,
#  truncation: copies keep a random 3' part of at least this fraction)
HUMAN_REPEATS = (
    ("alu", 0.10, (280, 320), 40, (0.02, 0.18), 1.0),        # SINE: ~1.2 M copies of ~300 bp
    ("l1", 0.17, (5500, 6500), 30, (0.03, 0.25), 0.1),       # LINE-1: mostly 5'-truncated
    ("l2_mir", 0.05, (150, 3000), 200, (0.15, 0.30), 0.2),  # old LINE-2 / MIR
    ("ltr", 0.08, (300, 8000), 300, (0.05, 0.25), 0.3),     # ERV / LTR elements
    ("dna", 0.03, (200, 2500), 200, (0.10, 0.30), 0.3),     # DNA transposons
)


def _scatter_copies(g: np.ndarray, fam: np.ndarray, n_copies: int, div_lo: float, div_hi: float, trunc: float,
                    rng: np.random.Generator) -> int:
    """Write n_copies diverged (and 5'-truncated) copies of fam at random
    positions of g, half of them reverse-complemented; vectorised per
    family.  Returns the bases written."""
    F = fam.size
    n = g.size
    if n_copies <= 0 or F >= n:
        return 0
    keep = np.maximum((F * (trunc + (1 - trunc) * rng.random(n_copies))).astype(np.int64), 1)
    div = div_lo + (div_hi - div_lo) * rng.random(n_copies)
    copies = np.broadcast_to(fam, (n_copies, F)).copy()
    hit = rng.random((n_copies, F)) < div[:, None]
    copies[hit] = (copies[hit] + rng.integers(1, 4, size=int(hit.sum()), dtype=np.uint8)) & 3
    rc = rng.random(n_copies) < 0.5
    copies[rc] = (3 - copies[rc])[:, ::-1]
    starts = (rng.random(n_copies) * (n - F)).astype(np.int64)
    # copy c keeps its last keep[c] bases (columns F-keep .. F-1 before the flip)
    col = np.arange(F)[None, :]
    mask = col >= (F - keep)[:, None]
    mask[rc] = mask[rc][:, ::-1]
    rows, cols = np.nonzero(mask)
    g[starts[rows] + cols] = copies[rows, cols]
    return int(keep.sum())


def _satellites(g: np.ndarray, frac: float, rng: np.random.Generator) -> None:
    """Alpha-satellite-like arrays (171-bp monomers, 2-10 % diverged, tens of
    kb long) and microsatellites (periods 1-6, 20-400 bp)."""
    n = g.size
    budget = int(n * frac * 0.8)
    mono = rng.integers(0, 4, size=171, dtype=np.uint8)
    while budget > 0 and n > 200_000:
        ln = int(rng.integers(20_000, 200_000))
        k = ln // 171 + 1
        arr = np.tile(mono, k)[:ln]
        hit = rng.random(ln) < float(rng.uniform(0.02, 0.10))
        arr[hit] = (arr[hit] + rng.integers(1, 4, size=int(hit.sum()), dtype=np.uint8)) & 3
        p = int(rng.integers(0, n - ln))
        g[p:p + ln] = arr
        budget -= ln
    budget = int(n * frac * 0.2)
    while budget > 0 and n > 20_000:
        m = min(4096, max(1, budget // 200))
        period = rng.integers(1, 7, size=m)
        ln = rng.integers(20, 400, size=m)
        for per, L in zip(period, ln):
            unit = rng.integers(0, 4, size=int(per), dtype=np.uint8)
            p = int(rng.integers(0, n - int(L)))
            g[p:p + int(L)] = np.resize(unit, int(L))
        budget -= int(ln.sum())


def make_genome_human_like(n_bp: int, seed: int = 1, n_chrom: int = 24, satellite_frac: float = 0.03) -> Genome:
    """Random genome with a human-like interspersed repeat profile (~46 % of
    the bases are repeat copies, HUMAN_REPEATS: Alu-like high-copy ~300-bp
    families at 2-18 % divergence, 5'-truncated ~6-kb L1-like families, old
    diverged LINE-2/MIR, LTR and DNA-transposon families) plus ~3 % satellite
    and simple-sequence arrays.  human_g1k_v37 is ~50 % repeats; the default
    make_genome has 2 %."""
    rng = np.random.default_rng([seed, 0x48554d])
    g = rng.integers(0, 4, size=n_bp, dtype=np.uint8)
    for _name, frac, (lo, hi), n_fam, (dlo, dhi), trunc in HUMAN_REPEATS:
        budget = int(n_bp * frac)
        fams = [rng.integers(0, 4, size=int(rng.integers(lo, hi + 1)), dtype=np.uint8) for _ in range(n_fam)]
        # family sizes in copy number follow a steep power law (a few very
        # young, high-copy families), the bases split accordingly
        w = 1.0 / np.arange(1, n_fam + 1) ** 1.2
        w /= w.sum()
        for f, share in zip(fams, w):
            mean_keep = f.size * (trunc + (1 - trunc) / 2)
            n_cp = int(budget * share / max(mean_keep, 1))
            while n_cp > 0:   # bounded temporaries: at most ~64 MB of copies at a time
                step = max(1, min(n_cp, (64 << 20) // f.size))
                _scatter_copies(g, f, step, dlo, dhi, trunc, rng)
                n_cp -= step
    _satellites(g, satellite_frac, rng)
    n_chrom = max(1, min(n_chrom, n_bp // 1000 if n_bp >= 1000 else 1))
    cuts = np.sort(rng.choice(np.arange(1, n_bp), size=n_chrom - 1, replace=False)) if n_chrom > 1 else np.array([], dtype=np.int64)
    starts = np.concatenate([[0], cuts, [n_bp]]).astype(np.int64)
    return Genome(g, [f"chr{i + 1}" for i in range(n_chrom)], starts)


def write_fasta(path: str, genome: Genome, width: int = 60) -> None:
    with open(path, "wb") as fh:
        for i, name in enumerate(genome.chrom_names):
            s = ACGT[genome.codes[genome.chrom_starts[i]:genome.chrom_starts[i + 1]]].tobytes()
            fh.write(b">" + name.encode() + b"\n")
            for k in range(0, len(s), width):
                fh.write(s[k:k + width] + b"\n")


def bns_contigs(n_bp: int, n_contigs: int = 24) -> list:
    """(name, offset, len) of n_contigs near-equal contigs chr1..chrN covering
    n_bp bases (each below 2^31: bntann1_t.len is an int32)."""
    n = max(1, min(n_contigs, n_bp))
    cuts = [n_bp * k // n for k in range(n + 1)]
    return [(f"chr{k + 1}", cuts[k], cuts[k + 1] - cuts[k]) for k in range(n)]


def write_bwa_bns(prefix: str, codes: np.ndarray, n_contigs: int = 24, chunk: int = 1 << 28) -> None:
    """The .pac / .ann / .amb `bwa index` writes for a genome of codes 0..3
    without ambiguous bases cut into bns_contigs (software/bntseq.c:63-93,
    :275-288): 2-bit forward strand, MSB first, then a 0 byte when l_pac % 4 == 0
    and l_pac % 4; contigs with gi 0, the "(null)" annotation bwa index gives a
    FASTA header without a comment, no holes; seed 11.  With
    the .bwt / .sa of the same codes these are a bwa index prefix (the FM
    index does not depend on where contigs start).  Streams the codes in
    chunks (a memory map of a human-size genome is fine)."""
    n = int(codes.size)
    with open(prefix + ".pac", "wb") as fh:
        for a in range(0, n, chunk):   # chunk is a multiple of 4
            c = np.minimum(np.asarray(codes[a:a + chunk], dtype=np.uint8), 3)
            pad = (-c.size) % 4
            if pad:
                c = np.concatenate([c, np.zeros(pad, np.uint8)])
            q = c.reshape(-1, 4)
            fh.write((q[:, 0] << 6 | q[:, 1] << 4 | q[:, 2] << 2 | q[:, 3]).astype(np.uint8).tobytes())
        if n % 4 == 0:
            fh.write(b"\0")
        fh.write(bytes([n % 4]))
    contigs = bns_contigs(n, n_contigs)
    with open(prefix + ".ann", "w") as fh:
        fh.write(f"{n} {len(contigs)} 11\n")
        for name, off, ln in contigs:
            fh.write(f"0 {name} (null)\n{off} {ln} 0\n")   # a FASTA line without comment
    with open(prefix + ".amb", "w") as fh:
        fh.write(f"{n} {len(contigs)} 0\n")


def write_fasta_contigs(path: str, codes: np.ndarray, n_contigs: int = 24, width: int = 60) -> None:
    """FASTA of codes cut as bns_contigs (what write_bwa_bns describes)."""
    with open(path, "wb") as fh:
        for name, off, ln in bns_contigs(int(codes.size), n_contigs):
            s = ACGT[np.minimum(codes[off:off + ln], 3)].tobytes()
            fh.write(b">" + name.encode() + b"\n")
            for k in range(0, len(s), width):
                fh.write(s[k:k + width] + b"\n")


def write_fastq(path: str, reads: "Reads", prefix: str = "r", qual: int = 40, pairs: bool = False) -> None:
    """Reads (codes 0..4) as FASTQ, named <prefix><index>; pairs: interleaved
    mates (make_pairs) named <prefix><index // 2>: bwa mem -p reads them as
    consecutive pairs (software/fastmap.c:65, 215) and names both mates alike."""
    sh = 1 if pairs else 0
    acgtn = np.frombuffer(b"ACGTN", dtype=np.uint8)
    q = chr(33 + qual)
    if reads.n and np.all(reads.lens == reads.lens[0]) and reads.lens[0] > 0:
        # fixed-length reads: the sequence lines in one array operation
        L = int(reads.lens[0])
        o = int(reads.offs[0])
        seqs = acgtn[np.minimum(reads.codes[o:o + reads.n * L], 4)].reshape(reads.n, L)
        qline = b"\n+\n" + (q * L).encode() + b"\n"
        with open(path, "wb") as fh:
            for i0 in range(0, reads.n, 65536):
                blk = seqs[i0:i0 + 65536]
                fh.write(b"".join(b"@%s%d\n%s%s" % (prefix.encode(), (i0 + k) >> sh, row.tobytes(), qline)
                                  for k, row in enumerate(blk)))
        return
    with open(path, "wb") as fh:
        for i in range(reads.n):
            s = acgtn[np.minimum(reads.read(i), 4)].tobytes()
            fh.write(b"@%s%d\n%s\n+\n%s\n" % (prefix.encode(), i >> sh, s, (q * len(s)).encode()))


def forward_reverse_text(codes: np.ndarray) -> np.ndarray:
    """The text BWA indexes: forward pac followed by its reverse complement
    (software/bntseq.c:303-309, bns_fasta2bntseq with for_only=0)."""
    return np.concatenate([codes, (3 - codes)[::-1]]).astype(np.uint8)


@dataclass
class Reads:
    lens: np.ndarray   # int32
    codes: np.ndarray  # uint8, concatenated
    offs: np.ndarray   # int64, n + 1

    @property
    def n(self) -> int:
        return int(self.lens.size)

    def read(self, i: int) -> np.ndarray:
        return self.codes[self.offs[i]:self.offs[i + 1]]

    def subset(self, idx) -> "Reads":
        idx = np.asarray(idx, dtype=np.int64)
        parts = [self.read(int(i)) for i in idx]
        lens = np.array([p.size for p in parts], dtype=np.int32)
        codes = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
        return Reads(lens, codes.astype(np.uint8), np.concatenate([[0], np.cumsum(lens, dtype=np.int64)]))


def make_reads(genome_codes: np.ndarray, n_reads: int, read_len, seed: int = 1, sub_rate: float = 0.02,
               n_rate: float = 0.001, revcomp_frac: float = 0.5, random_frac: float = 0.0) -> Reads:
    """Sample reads uniformly from the genome (both strands).

    read_len: an int (fixed) or a (lo, hi) tuple (uniform, inclusive).
    random_frac: fraction of reads replaced by unrelated random sequence.
    Substitutions at sub_rate, then ambiguous bases (code 4) at n_rate.
    """
    rng = np.random.default_rng(seed)
    G = genome_codes.size
    if isinstance(read_len, (tuple, list)):
        lens = rng.integers(read_len[0], read_len[1] + 1, size=n_reads).astype(np.int32)
    else:
        lens = np.full(n_reads, int(read_len), dtype=np.int32)
    lens = np.minimum(lens, min(G, 2**31 - 1)).astype(np.int32)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.int64)])
    total = int(offs[-1])
    codes = np.empty(total, dtype=np.uint8)
    if n_reads and np.all(lens == lens[0]) and lens[0] > 0:
        L = int(lens[0])
        pos = rng.integers(0, G - L + 1, size=n_reads)
        idx = pos[:, None] + np.arange(L)[None, :]
        mat = genome_codes[idx]
        rc = rng.random(n_reads) < revcomp_frac
        mat[rc] = (3 - mat[rc])[:, ::-1]
        codes[:] = mat.reshape(-1)
    else:
        pos = rng.integers(0, np.maximum(G - lens + 1, 1))
        rc = rng.random(n_reads) < revcomp_frac
        for i in range(n_reads):
            s = genome_codes[pos[i]:pos[i] + lens[i]]
            if rc[i]:
                s = (3 - s)[::-1]
            codes[offs[i]:offs[i + 1]] = s
    if random_frac > 0 and n_reads:
        rnd = np.nonzero(rng.random(n_reads) < random_frac)[0]
        for i in rnd:
            codes[offs[i]:offs[i + 1]] = rng.integers(0, 4, size=int(lens[i]), dtype=np.uint8)
    if sub_rate > 0 and total:
        hit = rng.random(total) < sub_rate
        codes[hit] = (codes[hit] + rng.integers(1, 4, size=int(hit.sum()), dtype=np.uint8)) & 3
    if n_rate > 0 and total:
        codes[rng.random(total) < n_rate] = 4
    return Reads(lens, codes, offs)


def block_seed(seed: int, b: int) -> int:
    """The seed of block b of a blocked read stream."""
    return int(np.random.SeedSequence([seed, b]).generate_state(1)[0])


def make_read_blocks(genome_codes: np.ndarray, blocks, block: int, read_len: int, seed: int = 1, pairs: bool = False,
                     **kw) -> Reads:
    """Blocks of a read stream defined block by block: block b holds `block`
    reads (pairs: block // 2 interleaved pairs) drawn with seed block_seed(seed, b),
    so any subset of blocks -- a rank's shard (contiguous
    chunks dealt round-robin to the GPUs) -- is generated without the rest,
    and shards reassembled in block order are the single-rank stream."""
    def one(b):
        s = block_seed(seed, int(b))
        if pairs:
            return make_pairs(genome_codes, block // 2, read_len, seed=s, **kw)
        return make_reads(genome_codes, block, read_len, seed=s, **kw)

    blocks = list(blocks)
    if len(blocks) > 2:   # blocks are independent: numpy releases the GIL in the bulk work
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=min(8, len(blocks))) as ex:
            parts = list(ex.map(one, blocks))
    else:
        parts = [one(b) for b in blocks]
    return concat_reads(parts) if parts else make_reads(genome_codes, 0, read_len, seed=seed)


def make_reads_big(genome_codes: np.ndarray, n_reads: int, read_len: int, seed: int = 1, block: int = 1 << 20,
                   **kw) -> Reads:
    """make_reads for read sets of tens of millions, generated in blocks of
    `block` reads (block b from block_seed(seed, b)) so one block's index
    matrix bounds the temporary memory; the last block is cut to n_reads."""
    nb = (n_reads + block - 1) // block
    r = make_read_blocks(genome_codes, range(nb), block, read_len, seed=seed, **kw)
    return r.subset(np.arange(n_reads)) if r.n > n_reads else r


def make_pairs(genome_codes: np.ndarray, n_pairs: int, read_len: int, seed: int = 1, insert_mean: float = 500.0,
               insert_sd: float = 50.0, sub_rate: float = 0.02, n_rate: float = 0.001, block: int = 1 << 19,
               with_pos: bool = False):
    """Paired-end reads, interleaved as bwa mem reads them (read 2k = mate 1,
    2k + 1 = mate 2 of pair k; software/bwamem.c:1600-1609): a fragment of
    length ~N(insert_mean, insert_sd) (at least read_len) from a uniform
    position; mate 1 is its first read_len bases, mate 2 the reverse
    complement of its last read_len bases (FR orientation); half of the
    fragments come from the reverse strand (mates swapped in effect).
    Substitutions at sub_rate and ambiguous bases at n_rate per base."""
    L = int(read_len)
    G = genome_codes.size
    lens = np.full(2 * n_pairs, L, dtype=np.int32)
    codes = np.empty(2 * n_pairs * L, dtype=np.uint8)
    frag = np.zeros((n_pairs, 3), dtype=np.int64)   # (start, insert, reverse strand)
    for b, a in enumerate(range(0, n_pairs, block)):
        n = min(block, n_pairs - a)
        rng = np.random.default_rng([seed, b])
        ins = np.clip(np.rint(rng.normal(insert_mean, insert_sd, size=n)), L, max(L, G - 1)).astype(np.int64)
        pos = (rng.random(n) * (G - ins + 1)).astype(np.int64)
        ar = np.arange(L)[None, :]
        m1 = genome_codes[pos[:, None] + ar]
        m2 = genome_codes[(pos + ins - L)[:, None] + ar]
        m2 = (3 - m2)[:, ::-1]
        rc = rng.random(n) < 0.5   # fragment from the reverse strand: mate 1 is the other end
        m1[rc], m2[rc] = m2[rc].copy(), m1[rc].copy()
        blk = np.empty((n, 2, L), dtype=np.uint8)
        blk[:, 0], blk[:, 1] = m1, m2
        flat = blk.reshape(-1)
        if sub_rate > 0:
            hit = rng.random(flat.size) < sub_rate
            flat[hit] = (flat[hit] + rng.integers(1, 4, size=int(hit.sum()), dtype=np.uint8)) & 3
        if n_rate > 0:
            flat[rng.random(flat.size) < n_rate] = 4
        codes[2 * a * L:2 * (a + n) * L] = flat
        frag[a:a + n, 0], frag[a:a + n, 1], frag[a:a + n, 2] = pos, ins, rc
    r = Reads(lens, codes, np.concatenate([[0], np.cumsum(lens, dtype=np.int64)]))
    return (r, frag) if with_pos else r


def concat_reads(parts) -> Reads:
    lens = np.concatenate([p.lens for p in parts]).astype(np.int32)
    codes = np.concatenate([p.codes for p in parts]).astype(np.uint8)
    return Reads(lens, codes, np.concatenate([[0], np.cumsum(lens, dtype=np.int64)]))


def write_smrd(path: str, reads: Reads) -> None:
    with open(path, "wb") as fh:
        fh.write(b"SMRD0001")
        fh.write(struct.pack("<QQ", reads.n, int(reads.codes.size)))
        fh.write(reads.lens.astype("<i4").tobytes())
        fh.write(reads.codes.astype(np.uint8).tobytes())


def read_smrd(path: str) -> Reads:
    with open(path, "rb") as fh:
        data = fh.read()
    if data[:8] != b"SMRD0001":
        raise ValueError(f"{path}: not an SMRD file")
    n, nb = struct.unpack_from("<QQ", data, 8)
    lens = np.frombuffer(data, dtype="<i4", count=n, offset=24).astype(np.int32)
    codes = np.frombuffer(data, dtype=np.uint8, count=nb, offset=24 + 4 * n).copy()
    return Reads(lens, codes, np.concatenate([[0], np.cumsum(lens, dtype=np.int64)]))


def read_smgo(path_or_bytes) -> list:
    """Parse an SMGO stream into [read][call] -> (n, 4) uint64 arrays."""
    if isinstance(path_or_bytes, (bytes, bytearray)):
        data = bytes(path_or_bytes)
    else:
        with open(path_or_bytes, "rb") as fh:
            data = fh.read()
    if data[:8] != b"SMGO0001":
        raise ValueError("not an SMGO stream")
    (n_reads,) = struct.unpack_from("<Q", data, 8)
    pos = 16
    out = []
    for _ in range(n_reads):
        (nc,) = struct.unpack_from("<I", data, pos)
        pos += 4
        calls = []
        for _ in range(nc):
            (n,) = struct.unpack_from("<I", data, pos)
            pos += 4
            arr = np.frombuffer(data, dtype="<u8", count=4 * n, offset=pos).reshape(n, 4).copy()
            pos += 32 * n
            calls.append(arr)
        out.append(calls)
    if pos != len(data):
        raise ValueError("trailing bytes in SMGO stream")
    return out


def read_smsa(path_or_bytes) -> list:
    """Parse an SMSA stream (include/smem_formats.h) into [read] -> uint64 positions."""
    if isinstance(path_or_bytes, (bytes, bytearray)):
        data = bytes(path_or_bytes)
    else:
        with open(path_or_bytes, "rb") as fh:
            data = fh.read()
    if data[:8] != b"SMSA0001":
        raise ValueError("not an SMSA stream")
    (n_reads,) = struct.unpack_from("<Q", data, 8)
    pos = 16
    out = []
    for _ in range(n_reads):
        (n,) = struct.unpack_from("<I", data, pos)
        pos += 4
        out.append(np.frombuffer(data, dtype="<u8", count=n, offset=pos).copy())
        pos += 8 * n
    if pos != len(data):
        raise ValueError("trailing bytes in SMSA stream")
    return out


def write_smsa(per_read) -> bytes:
    """SMSA stream bytes from [read] -> positions."""
    parts = [b"SMSA0001", struct.pack("<Q", len(per_read))]
    for p in per_read:
        p = np.ascontiguousarray(p, dtype="<u8")
        parts.append(struct.pack("<I", p.size))
        parts.append(p.tobytes())
    return b"".join(parts)


SEED_DT = np.dtype([("rbeg", "<i8"), ("qbeg", "<i4"), ("len", "<i4")])  # mem_seed_t


def read_smch(path_or_bytes) -> list:
    """Parse an SMCH stream (include/smem_formats.h) into [read] -> list of
    (pos, seeds) with seeds a SEED_DT array, in the stream's chain order."""
    if isinstance(path_or_bytes, (bytes, bytearray)):
        data = bytes(path_or_bytes)
    else:
        with open(path_or_bytes, "rb") as fh:
            data = fh.read()
    if data[:8] != b"SMCH0001":
        raise ValueError("not an SMCH stream")
    (n_reads,) = struct.unpack_from("<Q", data, 8)
    pos = 16
    out = []
    for _ in range(n_reads):
        (nc,) = struct.unpack_from("<I", data, pos)
        pos += 4
        chains = []
        for _ in range(nc):
            cpos, n = struct.unpack_from("<qI", data, pos)
            pos += 12
            chains.append((cpos, np.frombuffer(data, dtype=SEED_DT, count=n, offset=pos).copy()))
            pos += 16 * n
        out.append(chains)
    if pos != len(data):
        raise ValueError("trailing bytes in SMCH stream")
    return out


def write_smch(per_read) -> bytes:
    """SMCH stream bytes from [read] -> [(pos, seeds)]."""
    parts = [b"SMCH0001", struct.pack("<Q", len(per_read))]
    for chains in per_read:
        parts.append(struct.pack("<I", len(chains)))
        for cpos, seeds in chains:
            seeds = np.ascontiguousarray(seeds, dtype=SEED_DT)
            parts.append(struct.pack("<qI", int(cpos), seeds.size))
            parts.append(seeds.tobytes())
    return b"".join(parts)


# ---- SW extension tasks (ksw_extend2, software/ksw.c:379) ------------------
KSW_TASK = np.dtype([("q_off", "<u8"), ("t_off", "<u8"), ("qlen", "<i4"), ("tlen", "<i4"), ("w", "<i4"),
                     ("end_bonus", "<i4"), ("zdrop", "<i4"), ("h0", "<i4")])   # smem_ksw_task_t, 40 B
KSW_RESULT = np.dtype([(k, "<i4") for k in ("score", "qle", "tle", "gtle", "gscore", "max_off")])


def bwa_scmat(a: int = 1, b: int = 4) -> np.ndarray:
    """The m = 5 scoring matrix bwa_fill_scmat builds (software/bwa.c:84-93)."""
    m = np.full((5, 5), -1, dtype=np.int8)
    for i in range(4):
        for j in range(4):
            m[i, j] = a if i == j else -b
    return m.reshape(-1)


@dataclass
class KswBatch:
    tasks: np.ndarray   # KSW_TASK
    q: np.ndarray       # uint8 codes 0..4
    t: np.ndarray
    mat: np.ndarray     # int8[25]
    o_del: int = 6
    e_del: int = 1
    o_ins: int = 6
    e_ins: int = 1


def _mutated_copy(src: np.ndarray, rng, sub: float, indel: float) -> np.ndarray:
    out = []
    i = 0
    while i < src.size:
        r = rng.random()
        if r < indel / 2:            # insertion in the copy
            out.append(int(rng.integers(0, 4)))
            continue
        if r < indel:                # deletion from the copy
            i += 1
            continue
        c = int(src[i])
        if rng.random() < sub:
            c = (c + int(rng.integers(1, 4))) & 3
        out.append(c)
        i += 1
    return np.array(out, dtype=np.uint8)


def make_ksw_tasks(genome_codes: np.ndarray, n: int, seed: int = 1, max_qlen: int = 255) -> KswBatch:
    """Extension problems shaped like mem_chain2aln's (software/bwamem.c:1120-1170):
    from a seed inside a read sampled with substitutions and indels, the
    left extension (reversed prefix vs the reversed reference before the seed)
    and the right one (suffix vs the reference after it), the reference
    window padded by up to a band; plus unrelated sequences, N bases, tiny
    and empty problems, narrow / doubled bands, z-drop off."""
    rng = np.random.default_rng(seed)
    G = genome_codes
    tasks = np.zeros(n, dtype=KSW_TASK)
    qs, ts = [], []
    qo = to = 0
    for k in range(n):
        kind = rng.random()
        w = 100 if rng.random() < 0.8 else (200 if rng.random() < 0.5 else int(rng.integers(1, 21)))
        zdrop = 100 if rng.random() < 0.9 else (0 if rng.random() < 0.5 else int(rng.integers(1, 30)))
        end_bonus = 5 if rng.random() < 0.9 else int(rng.integers(0, 20))
        if kind < 0.04:     # tiny / empty
            qlen = int(rng.integers(1, 6))
            q = rng.integers(0, 5, size=qlen).astype(np.uint8)
            t = rng.integers(0, 5, size=int(rng.integers(0, 6))).astype(np.uint8)
            h0 = int(rng.integers(0, 40))
        elif kind < 0.12:   # unrelated
            qlen = int(rng.integers(1, max_qlen + 1))
            q = rng.integers(0, 4, size=qlen).astype(np.uint8)
            t = rng.integers(0, 4, size=int(rng.integers(0, qlen + 120))).astype(np.uint8)
            h0 = int(rng.integers(0, 80))
        else:
            L = int(rng.choice([100, 150, 250]))
            pos = int(rng.integers(300, G.size - L - 600))
            ref = G[pos - 250:pos + L + 250]
            read = _mutated_copy(G[pos:pos + L], rng, float(rng.choice([0.0, 0.02, 0.05])), 0.004)
            if rng.random() < 0.1:
                read[rng.random(read.size) < 0.02] = 4
            if read.size < 30:
                read = G[pos:pos + L].copy()
            sl = int(rng.integers(19, min(60, read.size - 1)))
            q0 = int(rng.integers(0, read.size - sl + 1))
            pad = int(rng.integers(0, 110))
            if rng.random() < 0.5:  # left extension: reversed prefix, reversed reference before the seed
                q = read[:q0][::-1].copy()
                r0 = 250 + q0
                t = ref[max(0, r0 - q0 - pad):r0][::-1].copy()
                h0 = sl
            else:                    # right extension: suffix after the seed
                q = read[q0 + sl:].copy()
                r0 = 250 + q0 + sl
                t = ref[r0:r0 + q.size + pad].copy()
                h0 = int(rng.integers(sl, sl + 120))
            if q.size == 0:
                q = read[:1].copy()
            q = q[:max_qlen]
            qlen = q.size
        tasks[k] = (qo, to, qlen, t.size, w, end_bonus, zdrop, h0)
        qs.append(q)
        ts.append(t)
        qo += q.size
        to += t.size
    qpool = np.concatenate(qs).astype(np.uint8) if qs else np.zeros(0, np.uint8)
    tpool = np.concatenate(ts).astype(np.uint8) if ts else np.zeros(0, np.uint8)
    return KswBatch(tasks, qpool, tpool, bwa_scmat())


def write_smkt(path: str, b: KswBatch) -> None:
    with open(path, "wb") as fh:
        fh.write(b"SMKT0001")
        fh.write(struct.pack("<QQQ", b.tasks.size, b.q.size, b.t.size))
        fh.write(np.asarray(b.mat, dtype=np.int8).tobytes() + b"\0\0\0")
        fh.write(struct.pack("<4i", b.o_del, b.e_del, b.o_ins, b.e_ins))
        fh.write(b.tasks.astype(KSW_TASK).tobytes())
        fh.write(b.q.astype(np.uint8).tobytes())
        fh.write(b.t.astype(np.uint8).tobytes())


def read_smkt(data: bytes) -> KswBatch:
    if data[:8] != b"SMKT0001":
        raise ValueError("not an SMKT file")
    n, qb, tb = struct.unpack_from("<QQQ", data, 8)
    o = 32
    mat = np.frombuffer(data, dtype=np.int8, count=25, offset=o).copy()
    o += 28
    o_del, e_del, o_ins, e_ins = struct.unpack_from("<4i", data, o)
    o += 16
    tasks = np.frombuffer(data, dtype=KSW_TASK, count=n, offset=o).copy()
    o += n * KSW_TASK.itemsize
    q = np.frombuffer(data, dtype=np.uint8, count=qb, offset=o).copy()
    o += qb
    t = np.frombuffer(data, dtype=np.uint8, count=tb, offset=o).copy()
    return KswBatch(tasks, q, t, mat, o_del, e_del, o_ins, e_ins)


def read_smkr(data: bytes) -> np.ndarray:
    if data[:8] != b"SMKR0001":
        raise ValueError("not an SMKR file")
    (n,) = struct.unpack_from("<Q", data, 8)
    return np.frombuffer(data, dtype=KSW_RESULT, count=n, offset=16).copy()


# ---- ksw_align2 problems (mem_chain2aln_short, software/bwamem.c:805-852) ----
KSWA_TASK = np.dtype([("q_off", "<u8"), ("t_off", "<u8"), ("qlen", "<i4"), ("tlen", "<i4"), ("xtra", "<i4"),
                      ("pad", "<i4")])   # smem_ksw_atask_t, 32 B
KSWA_RESULT = np.dtype([(k, "<i4") for k in ("score", "te", "qe", "score2", "te2", "tb", "qb")])  # kswr_t
KSW_XBYTE, KSW_XSTOP, KSW_XSUBO, KSW_XSTART = 0x10000, 0x20000, 0x40000, 0x80000


def make_kswa_tasks(genome_codes: np.ndarray, n: int, seed: int = 1, a: int = 1, b: int = 4, o: int = 6, e: int = 1,
                    min_seed_len: int = 19) -> "KswBatch":
    """ksw_align2 problems shaped like mem_chain2aln_short's: the query span of a
    chain plus MEM_SHORT_EXT = 50 on both sides (< 200 bp) against the
    reference span of its seeds plus 50 (lengths within 50 of each other),
    with substitutions, small indels and Ns; xtra = KSW_XSUBO | KSW_XSTART |
    (KSW_XBYTE when qlen * a < 250) | min_seed_len * a, as software/bwamem.c:835.
    Some problems are unrelated sequence, tiny, or run with other flag sets
    (no start pass, no suboptimal threshold, a threshold above the score)."""
    rng = np.random.default_rng(seed)
    G = genome_codes
    tasks = np.zeros(n, dtype=KSWA_TASK)
    qs, ts = [], []
    qo = to = 0
    for k in range(n):
        kind = rng.random()
        if kind < 0.05:      # tiny
            q = rng.integers(0, 5, size=int(rng.integers(1, 8))).astype(np.uint8)
            t = rng.integers(0, 5, size=int(rng.integers(0, 10))).astype(np.uint8)
        elif kind < 0.15:    # unrelated
            q = rng.integers(0, 4, size=int(rng.integers(20, 200))).astype(np.uint8)
            t = rng.integers(0, 4, size=int(rng.integers(0, 250))).astype(np.uint8)
        else:
            ql = int(rng.integers(60, 200))
            pos = int(rng.integers(300, G.size - ql - 300))
            read = _mutated_copy(G[pos:pos + ql], rng, float(rng.choice([0.0, 0.01, 0.03, 0.06])),
                                 float(rng.choice([0.0, 0.005, 0.02])))[:199]
            if rng.random() < 0.15:
                read[rng.random(read.size) < 0.02] = 4
            d = int(rng.integers(-50, 51))
            lo = pos - int(rng.integers(0, 40))
            t = G[lo:lo + max(1, min(256, read.size + d + (pos - lo)))].copy()
            q = read if read.size else G[pos:pos + 1].copy()
            if rng.random() < 0.3:   # the reverse strand
                q = np.where(q < 4, 3 - q, 4)[::-1].astype(np.uint8)
                t = (3 - t)[::-1].astype(np.uint8)
        q = q[:199] if q.size else np.zeros(1, np.uint8)
        t = t[:256]
        xtra = KSW_XSUBO | KSW_XSTART | (KSW_XBYTE if q.size * a < 250 else 0) | (min_seed_len * a)
        r = rng.random()
        if r < 0.05:
            xtra &= ~KSW_XSTART
        elif r < 0.10:
            xtra = KSW_XSTART | (KSW_XBYTE if q.size * a < 250 else 0)
        elif r < 0.13:
            xtra = KSW_XSUBO | KSW_XSTART | (KSW_XBYTE if q.size * a < 250 else 0) | 200
        tasks[k] = (qo, to, q.size, t.size, xtra, 0)
        qs.append(q)
        ts.append(t)
        qo += q.size
        to += t.size
    qpool = np.concatenate(qs).astype(np.uint8) if qs else np.zeros(0, np.uint8)
    tpool = np.concatenate(ts).astype(np.uint8) if ts else np.zeros(0, np.uint8)
    return KswBatch(tasks, qpool, tpool, bwa_scmat(a, b), o, e, o, e)


def write_smat(path: str, b: "KswBatch") -> None:
    with open(path, "wb") as fh:
        fh.write(b"SMAT0001")
        fh.write(struct.pack("<QQQ", b.tasks.size, b.q.size, b.t.size))
        fh.write(np.asarray(b.mat, dtype=np.int8).tobytes() + b"\0\0\0")
        fh.write(struct.pack("<4i", b.o_del, b.e_del, b.o_ins, b.e_ins))
        fh.write(b.tasks.astype(KSWA_TASK).tobytes())
        fh.write(b.q.astype(np.uint8).tobytes())
        fh.write(b.t.astype(np.uint8).tobytes())


def read_smat(data: bytes) -> "KswBatch":
    if data[:8] != b"SMAT0001":
        raise ValueError("not an SMAT file")
    n, qb, tb = struct.unpack_from("<QQQ", data, 8)
    o = 32
    mat = np.frombuffer(data, dtype=np.int8, count=25, offset=o).copy()
    o += 28
    o_del, e_del, o_ins, e_ins = struct.unpack_from("<4i", data, o)
    o += 16
    tasks = np.frombuffer(data, dtype=KSWA_TASK, count=n, offset=o).copy()
    o += n * KSWA_TASK.itemsize
    q = np.frombuffer(data, dtype=np.uint8, count=qb, offset=o).copy()
    o += qb
    t = np.frombuffer(data, dtype=np.uint8, count=tb, offset=o).copy()
    return KswBatch(tasks, q, t, mat, o_del, e_del, o_ins, e_ins)


def read_smar(data: bytes) -> np.ndarray:
    if data[:8] != b"SMAR0001":
        raise ValueError("not an SMAR file")
    (n,) = struct.unpack_from("<Q", data, 8)
    return np.frombuffer(data, dtype=KSWA_RESULT, count=n, offset=16).copy()

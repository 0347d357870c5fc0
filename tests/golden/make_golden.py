"""Regenerate the committed golden fixtures from the compiled reference.

    python tests/golden/make_golden.py

Needs oracle/_ref/ref_harness (built by `make -C oracle ref`, which compiles
the reference's own C sources in place from /root/reference/software).
Inputs are seeded synthetic data; every output file here is produced by the
reference code itself:

  g1.fa.gz            genome (300 kbp, 4 records, repeat families / exact / tandem repeats)
  g1.bwt.gz           `bwa index -a is` of g1.fa   (software/bwtindex.c:187)
  r1.smrd.gz          1500 reads (SMRD, include/smem_formats.h), mixed shapes
  g1_<case>.smgo.gz   reference smem_next2 streams under mem_insert_seed
                      (software/bwamem.c:453-460) for each option set
  g1.sa.gz            the `bwa index` sampled suffix array (.sa, software/bwt.c:852)
  g1_<case>.smsa.gz   reference bwt_sa() of every seed occurrence of that stream
                      (software/bwamem.c:467-474, max_occ 10000)
  manifest.json       cases, options, sha256 of the uncompressed streams
"""
import gzip
import hashlib
import json
import os
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)

from smemgpu import synth  # noqa: E402
from oracle import oracle  # noqa: E402

MAX_OCC = 10000  # mem_opt_t.max_occ default of this reference (software/bwamem.c:60)

CASES = [
    dict(name="default", n_reads=1500, opt=dict(min_seed_len=19, split_factor=1.5, split_width=10, start_width=1)),
    dict(name="noexact", n_reads=500, opt=dict(min_seed_len=19, split_factor=1.5, split_width=10, start_width=2)),
    dict(name="k14s20", n_reads=500, opt=dict(min_seed_len=14, split_factor=1.5, split_width=20, start_width=1)),
    dict(name="reseed", n_reads=500, opt=dict(min_seed_len=19, split_factor=1.0, split_width=500, start_width=1)),
    dict(name="k30", n_reads=500, opt=dict(min_seed_len=30, split_factor=2.0, split_width=3, start_width=1)),
]


def make_reads(g):
    parts = [
        synth.make_reads(g, 500, 150, seed=101),
        synth.make_reads(g, 200, 100, seed=102),
        synth.make_reads(g, 200, 250, seed=103),
        synth.make_reads(g, 200, 150, seed=104, sub_rate=0.05),
        synth.make_reads(g, 200, (1, 320), seed=105, n_rate=0.02),
        synth.make_reads(g, 100, 101, seed=106, random_frac=1.0),
        synth.make_reads(g, 100, (10, 40), seed=107),
    ]
    r = synth.concat_reads(parts)
    perm = np.random.default_rng(108).permutation(r.n)
    return r.subset(perm)


def gz_write(path, data: bytes):
    with gzip.GzipFile(path, "wb", mtime=0) as fh:
        fh.write(data)


def main():
    if not oracle.ref_available():
        oracle.build(ref=True)
    tmp = tempfile.mkdtemp()
    try:
        genome = synth.make_genome(300_000, seed=11)
        fa = os.path.join(tmp, "g1.fa")
        synth.write_fasta(fa, genome)
        oracle.ref_index(fa, os.path.join(tmp, "g1"))
        reads = make_reads(genome.codes)
        smrd = os.path.join(tmp, "r1.smrd")
        synth.write_smrd(smrd, reads)
        with open(fa, "rb") as fh:
            gz_write(os.path.join(HERE, "g1.fa.gz"), fh.read())
        with open(os.path.join(tmp, "g1.bwt"), "rb") as fh:
            gz_write(os.path.join(HERE, "g1.bwt.gz"), fh.read())
        with open(os.path.join(tmp, "g1.sa"), "rb") as fh:
            gz_write(os.path.join(HERE, "g1.sa.gz"), fh.read())
        with open(smrd, "rb") as fh:
            gz_write(os.path.join(HERE, "r1.smrd.gz"), fh.read())
        manifest = {"genome": dict(n_bp=300_000, seed=11), "cases": []}
        for case in CASES:
            sub = reads.subset(np.arange(case["n_reads"]))
            p = os.path.join(tmp, "sub.smrd")
            synth.write_smrd(p, sub)
            out = os.path.join(tmp, case["name"] + ".smgo")
            oracle.ref_smem(os.path.join(tmp, "g1.bwt"), p, out, **case["opt"])
            with open(out, "rb") as fh:
                data = fh.read()
            gz_write(os.path.join(HERE, f"g1_{case['name']}.smgo.gz"), data)
            parsed = synth.read_smgo(data)
            sa_out = os.path.join(tmp, case["name"] + ".smsa")
            oracle.ref_sa(os.path.join(tmp, "g1.bwt"), os.path.join(tmp, "g1.sa"), out, sa_out,
                          min_seed_len=case["opt"]["min_seed_len"], max_occ=MAX_OCC)
            with open(sa_out, "rb") as fh:
                sa_data = fh.read()
            gz_write(os.path.join(HERE, f"g1_{case['name']}.smsa.gz"), sa_data)
            manifest["cases"].append(dict(case, sha256=hashlib.sha256(data).hexdigest(),
                                          n_intv=int(sum(a.shape[0] for r in parsed for a in r)),
                                          n_calls=int(sum(len(r) for r in parsed)),
                                          max_occ=MAX_OCC, sa_sha256=hashlib.sha256(sa_data).hexdigest(),
                                          n_occ=int(sum(p.size for p in synth.read_smsa(sa_data)))))
        with open(os.path.join(HERE, "manifest.json"), "w") as fh:
            json.dump(manifest, fh, indent=1)
        print(json.dumps(manifest, indent=1))
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    main()

"""Golden SAM from the unpatched reference pipeline (end-to-end parity of the
reference-side binding, integration/).

    python tests/golden/make_golden_sam.py

For g1 (300 kbp) and g2 (150 kbp, repeat-dense) of the committed fixtures:
  sam/<g>_se.fq.gz   single-end reads: the committed SMRD reads (r1 / r2) of
                     at least 30 bp (shorter ones hit an out-of-bounds read of
                     the reference's batched path, software/bwamem.c:387
                     itr[batch_size]->len, when len <= split_len), as FASTQ
  sam/<g>_pe.fq.gz   interleaved pairs (synth.make_pairs: 150 bp, insert N(500, 50))
  sam/<g>_<se|pe>.sam.gz
                     `bwa mem -t 1 -b 1` of the reference (oracle/_ref/ref_harness
                     mem: main_mem's body over mem_process_seqs, every batch on
                     bwt_smem1_batched's CPU path), index by the reference's own
                     `bwa index -a is`; the @PG line is the harness's.
"""
import gzip
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)

from smemgpu import synth  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
OUT = os.path.join(HERE, "sam")
QUAL = 40


def write_fastq(path: str, reads, names) -> None:
    acgtn = np.frombuffer(b"ACGTN", dtype=np.uint8)
    with gzip.open(path, "wb", compresslevel=9) as fh:
        for i in range(reads.n):
            s = acgtn[np.minimum(reads.read(i), 4)].tobytes()
            q = bytes([33 + QUAL]) * len(s)
            fh.write(b"@" + names[i].encode() + b"\n" + s + b"\n+\n" + q + b"\n")


def genome_codes(fa_gz: str) -> np.ndarray:
    seq = []
    with gzip.open(fa_gz, "rb") as fh:
        for line in fh:
            if not line.startswith(b">"):
                seq.append(line.strip())
    return synth.NT4[np.frombuffer(b"".join(seq), dtype=np.uint8)]


def main():
    os.makedirs(OUT, exist_ok=True)
    man = {}
    with tempfile.TemporaryDirectory() as d:
        for g, rfile, pseed in (("g1", "r1.smrd.gz", 11), ("g2", "r2.smrd.gz", 12)):
            fa = os.path.join(d, g + ".fa")
            with gzip.open(os.path.join(HERE, g + ".fa.gz"), "rb") as src, open(fa, "wb") as dst:
                shutil.copyfileobj(src, dst)
            subprocess.run([REF, "index", fa, fa], check=True, capture_output=True)
            smrd = os.path.join(d, "r.smrd")
            with gzip.open(os.path.join(HERE, rfile), "rb") as src, open(smrd, "wb") as dst:
                shutil.copyfileobj(src, dst)
            r = synth.read_smrd(smrd)
            keep = np.nonzero(r.lens >= 30)[0]
            se = r.subset(keep)
            pe = synth.make_pairs(genome_codes(os.path.join(HERE, g + ".fa.gz")), 300, 150, seed=pseed,
                                  sub_rate=0.02, n_rate=0.002)
            for kind, reads, names, is_pe in (("se", se, [f"r{int(i)}" for i in keep], 0),
                                              ("pe", pe, [f"p{k // 2}" for k in range(pe.n)], 1)):
                fq = os.path.join(OUT, f"{g}_{kind}.fq.gz")
                write_fastq(fq, reads, names)
                p = subprocess.run([REF, "mem", fa, fq, "1", "1", str(is_pe)], check=True, capture_output=True)
                with gzip.open(os.path.join(OUT, f"{g}_{kind}.sam.gz"), "wb", compresslevel=9) as fh:
                    fh.write(p.stdout)
                body = b"".join(l + b"\n" for l in p.stdout.split(b"\n") if l and not l.startswith(b"@PG"))
                man[f"{g}_{kind}"] = {"reads": int(reads.n), "sam_lines": body.count(b"\n"),
                                      "sha256_sam_without_pg": hashlib.sha256(body).hexdigest()}
                print(g, kind, man[f"{g}_{kind}"], flush=True)
    with open(os.path.join(OUT, "manifest.json"), "w") as fh:
        json.dump(man, fh, indent=1)


if __name__ == "__main__":
    main()

"""Loader for the committed golden fixtures (tests/golden/, made by
tests/golden/make_golden.py from the compiled reference)."""
import gzip
import hashlib
import json
import os
from dataclasses import dataclass

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _gz(name: str) -> bytes:
    with gzip.open(os.path.join(GOLDEN, name), "rb") as fh:
        return fh.read()


def fasta_codes(data: bytes) -> np.ndarray:
    from smemgpu import synth
    seq = b"".join(line for line in data.split(b"\n") if line and not line.startswith(b">"))
    return synth.NT4[np.frombuffer(seq, dtype=np.uint8)]


@dataclass
class Fixture:
    manifest: dict
    genome: np.ndarray
    bwt_bytes: bytes
    reads: object
    index: object

    @property
    def cases(self):
        return self.manifest["cases"]

    def stream(self, case) -> bytes:
        data = _gz(f"g1_{case['name']}.smgo.gz")
        assert hashlib.sha256(data).hexdigest() == case["sha256"], "fixture corrupted"
        return data

    @property
    def sa_bytes(self) -> bytes:
        """the reference `bwa index` .sa of the golden genome"""
        return _gz("g1.sa.gz")

    def sa_stream(self, case) -> bytes:
        """reference bwt_sa of every seed occurrence of the case's stream (SMSA)"""
        data = _gz(f"g1_{case['name']}.smsa.gz")
        assert hashlib.sha256(data).hexdigest() == case["sa_sha256"], "fixture corrupted"
        return data


_cache = None


def load() -> Fixture:
    global _cache
    if _cache is None:
        import tempfile
        import smemgpu
        from smemgpu import synth
        with open(os.path.join(GOLDEN, "manifest.json")) as fh:
            manifest = json.load(fh)
        genome = fasta_codes(_gz("g1.fa.gz"))
        bwt_bytes = _gz("g1.bwt.gz")
        with tempfile.TemporaryDirectory() as d:
            p = os.path.join(d, "r1.smrd")
            with open(p, "wb") as fh:
                fh.write(_gz("r1.smrd.gz"))
            reads = synth.read_smrd(p)
            b = os.path.join(d, "g1.bwt")
            with open(b, "wb") as fh:
                fh.write(bwt_bytes)
            index = smemgpu.Index.read(b)
        _cache = Fixture(manifest, genome, bwt_bytes, reads, index)
    return _cache


# ------------------------------------------------------------ chains (+ g2)
def gz(name: str) -> bytes:
    return _gz(name)


def genome_cases(genome: str):
    """the seeding cases of a golden genome ("g1" or the repeat-dense "g2")"""
    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        m = json.load(fh)
    return m["cases"] if genome == "g1" else m["g2"]["cases"]


def chain_fixtures():
    """every (genome, seeding case, chain option set + filter) with a reference
    SMCH stream"""
    out = []
    for g in ("g1", "g2"):
        for c in genome_cases(g):
            for ch in c.get("chains", []):
                out.append((g, c, ch))
    return out


def l_pac(genome: str) -> int:
    import struct
    return struct.unpack_from("<5Q", _gz(f"{genome}.bwt.gz"), 0)[4] // 2


def smgo(genome: str, case) -> bytes:
    data = _gz(f"{genome}_{case['name']}.smgo.gz")
    assert hashlib.sha256(data).hexdigest() == case["sha256"], "fixture corrupted"
    return data


def smsa(genome: str, case) -> bytes:
    data = _gz(f"{genome}_{case['name']}.smsa.gz")
    assert hashlib.sha256(data).hexdigest() == case["sa_sha256"], "fixture corrupted"
    return data


def smch(chain) -> bytes:
    data = _gz(chain["file"])
    assert hashlib.sha256(data).hexdigest() == chain["sha256"], "fixture corrupted"
    return data


def files(genome: str, d: str):
    """write the genome's .bwt / .sa / reads into directory d; returns the paths"""
    reads = "r1.smrd" if genome == "g1" else "r2.smrd"
    out = {}
    for name in (f"{genome}.bwt", f"{genome}.sa", reads):
        p = os.path.join(d, name)
        with open(p, "wb") as fh:
            fh.write(_gz(name + ".gz"))
        out[name.split(".")[-1]] = p
    return out

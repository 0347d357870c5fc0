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


# ---- chains -> regions (mem_chain2aln) fixtures ----------------------------
ALNREG_DT = np.dtype([("rb", "<i8"), ("re", "<i8"), ("qb", "<i4"), ("qe", "<i4"), ("score", "<i4"),
                      ("truesc", "<i4"), ("sub", "<i4"), ("csub", "<i4"), ("sub_n", "<i4"), ("w", "<i4"),
                      ("seedcov", "<i4"), ("secondary", "<i4"), ("hash", "<u8")])   # smem_alnreg_t, 64 B
_SMRG_REC = np.dtype([("rb", "<i8"), ("re", "<i8"), ("qb", "<i4"), ("qe", "<i4"), ("score", "<i4"),
                      ("truesc", "<i4"), ("sub", "<i4"), ("csub", "<i4"), ("sub_n", "<i4"), ("w", "<i4"),
                      ("seedcov", "<i4"), ("secondary", "<i4")])


def aln_fixtures():
    """every (genome, seeding case, chain file, region file) the reference's
    mem_chain2aln loop produced (tests/golden/make_golden.py make_aln)"""
    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        return json.load(fh).get("aln", [])


def pac(genome: str) -> np.ndarray:
    """the 2-bit forward strand bwa_index wrote (software/bntseq.c:303-309)"""
    n = (l_pac(genome) + 3) // 4
    return np.frombuffer(_gz(f"{genome}.pac.gz"), dtype=np.uint8)[:n].copy()


def smch_parse(data: bytes):
    """SMCH stream -> (chains as smemgpu CHAIN_DT, chain_off[n+1], seeds as SEED_DT)"""
    import struct
    from smemgpu.lib import CHAIN_DT, SEED_DT
    assert data[:8] == b"SMCH0001"
    n_reads = struct.unpack_from("<Q", data, 8)[0]
    p, chains, seeds, off = 16, [], [], [0]
    for _ in range(n_reads):
        nc = struct.unpack_from("<I", data, p)[0]
        p += 4
        for _ in range(nc):
            pos, n = struct.unpack_from("<qI", data, p)
            p += 12
            chains.append((pos, len(seeds), n, 0))
            for _ in range(n):
                seeds.append(struct.unpack_from("<qii", data, p))
                p += 16
        off.append(len(chains))
    return (np.array(chains, dtype=CHAIN_DT), np.array(off, dtype=np.uint64), np.array(seeds, dtype=SEED_DT))


def smrg_parse(data: bytes):
    """SMRG stream -> (regions as ALNREG_DT, reg_off[n+1])"""
    import struct
    assert data[:8] == b"SMRG0001"
    n_reads = struct.unpack_from("<Q", data, 8)[0]
    p, parts, off = 16, [], [0]
    for _ in range(n_reads):
        n = struct.unpack_from("<I", data, p)[0]
        p += 4
        parts.append(np.frombuffer(data, dtype=_SMRG_REC, count=n, offset=p))
        p += n * _SMRG_REC.itemsize
        off.append(off[-1] + n)
    regs = np.zeros(off[-1], dtype=ALNREG_DT)
    if off[-1]:
        cat = np.concatenate(parts)
        for f in _SMRG_REC.names:
            regs[f] = cat[f]
    return regs, np.array(off, dtype=np.uint64)


def smrg(fix) -> bytes:
    data = _gz(fix["file"])
    assert hashlib.sha256(data).hexdigest() == fix["sha256"], "fixture corrupted"
    return data

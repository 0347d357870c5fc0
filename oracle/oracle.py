"""TEST INFRASTRUCTURE ONLY — ctypes binding of the C restatement
(oracle/smem_oracle.c -> oracle/_build/liboracle.so) and of the compiled
reference harness (oracle/_ref/ref_harness).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module; the product never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
CLI = os.path.join(HERE, "_build", "smem_oracle")
REF = os.path.join(HERE, "_ref", "ref_harness")
REF_SRC = "/root/reference/software"


def build(ref: bool = True) -> None:
    """Compile the restatement, and the reference harness when /root/reference exists."""
    subprocess.run(["make", "-s", "-C", HERE, "port"], check=True)
    if ref and os.path.isdir(REF_SRC):
        subprocess.run(["make", "-s", "-C", HERE, "ref", "-j8"], check=True)


class OptT(C.Structure):
    _fields_ = [("min_seed_len", C.c_int), ("split_factor", C.c_float), ("split_width", C.c_int),
                ("start_width", C.c_int)]


class Stats(C.Structure):
    _fields_ = [(k, C.c_uint64) for k in ("n_calls", "n_intv", "n_smem1", "n_ext", "n_ext_ref", "n_bkt",
                                          "n_bkt_ref", "n_bases", "n_bkt64", "n_ext_fwd",
                                          "n_ext_u1_fwd", "n_ext_u1_bwd", "n_run_u1", "n_ext_fwd_k12")] + [
        ("n_ext_len", C.c_uint64 * 33), ("n_fwd_push", C.c_uint64), ("n_bwd_push_hi", C.c_uint64),
        ("n_bwd_read_hi", C.c_uint64), ("n_fwd_spill", C.c_uint64),
        ("n_bwd_step", C.c_uint64), ("n_step_hist", C.c_uint64 * 17), ("n_bwd_task_hi", C.c_uint64),
        ("n_tm_saved", C.c_uint64), ("n_tm_sa", C.c_uint64), ("n_tm_isa", C.c_uint64), ("n_tm_runs", C.c_uint64),
        ("n_tm_bases", C.c_uint64)]

    def as_dict(self) -> dict:
        return {k: (list(getattr(self, k)) if k in ("n_ext_len", "n_step_hist") else int(getattr(self, k))) for k, _ in self._fields_}


class ChainOptT(C.Structure):
    _fields_ = [("w", C.c_int), ("max_chain_gap", C.c_int), ("min_seed_len", C.c_int), ("mask_level", C.c_float),
                ("drop_ratio", C.c_float), ("filter", C.c_int)]


class KswOptT(C.Structure):
    _fields_ = [("mat", C.c_int8 * 25), ("pad", C.c_int8 * 3), ("o_del", C.c_int32), ("e_del", C.c_int32),
                ("o_ins", C.c_int32), ("e_ins", C.c_int32)]


_lib = None


def load() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build(ref=False)
        lib = C.CDLL(LIB)
        lib.orc_bwt_load.argtypes = [C.c_char_p]
        lib.orc_bwt_load.restype = C.c_void_p
        lib.orc_bwt_wrap.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64)]
        lib.orc_bwt_wrap.restype = C.c_void_p
        lib.orc_bwt_free.argtypes = [C.c_void_p]
        lib.orc_bwt_free.restype = None
        lib.orc_seed.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.POINTER(OptT), C.c_int,
                                 C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_uint64), C.c_void_p, C.c_void_p,
                                 C.c_void_p, C.POINTER(Stats)]
        lib.orc_seed_timed.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.POINTER(OptT), C.c_int,
                                       C.POINTER(Stats)]
        lib.orc_seed_timed.restype = C.c_double
        lib.orc_seed_trace.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.POINTER(OptT), C.c_void_p,
                                       C.c_uint64, C.c_void_p]
        lib.orc_seed_trace.restype = C.c_int64
        lib.orc_free.argtypes = [C.c_void_p]
        lib.orc_free.restype = None
        lib.orc_occ4.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
        lib.orc_occ4.restype = None
        lib.orc_sa_load.argtypes = [C.c_char_p]
        lib.orc_sa_load.restype = C.c_void_p
        lib.orc_sa_wrap.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64]
        lib.orc_sa_wrap.restype = C.c_void_p
        lib.orc_sa_free.argtypes = [C.c_void_p]
        lib.orc_sa_free.restype = None
        lib.orc_sa_lookup.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        lib.orc_sa_lookup.restype = C.c_uint64
        lib.orc_sa_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_int]
        lib.orc_sa_batch.restype = None
        lib.orc_ksw_batch.argtypes = [C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(KswOptT), C.c_void_p]
        lib.orc_ksw_batch.restype = C.c_int
        lib.orc_chain.argtypes = [C.c_int64, C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(ChainOptT), C.c_int,
                                  C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_uint64)]
        lib.orc_aln_batch.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p), C.c_void_p]
        lib.orc_aln_batch.restype = C.c_int
        lib.orc_cells.argtypes = [C.POINTER(C.c_uint64), C.c_int]
        lib.orc_cells.restype = None
        lib.orc_ext_shapes.argtypes = [C.POINTER(C.c_uint64), C.c_int]
        lib.orc_ext_shapes.restype = None
        lib.orc_seed_uses.argtypes = [C.POINTER(C.c_uint64), C.c_int]
        lib.orc_seed_uses.restype = None
        lib.orc_ksw_align2.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                       C.c_int, C.c_int, C.POINTER(C.c_int32)]
        lib.orc_ksw_align2.restype = None
        _lib = lib
    return _lib


class OracleIndex:
    def __init__(self, path: str | None = None, words=None, primary=None, L2=None):
        lib = load()
        if path is not None:
            self._h = lib.orc_bwt_load(path.encode())
            if not self._h:
                raise IOError(path)
            self._keep = None
        else:
            w = np.ascontiguousarray(words, dtype=np.uint32)
            self._keep = w
            l2 = (C.c_uint64 * 5)(*[int(v) for v in L2])
            self._h = lib.orc_bwt_wrap(w.ctypes.data, w.size, int(primary), l2)

    def occ4(self, k: int) -> np.ndarray:
        out = (C.c_uint64 * 4)()
        load().orc_occ4(self._h, C.c_uint64(k & 0xFFFFFFFFFFFFFFFF), out)
        return np.array(list(out), dtype=np.uint64)

    def close(self):
        if self._h:
            load().orc_bwt_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class OracleSA:
    """Sampled SA (bwa's .sa: sa[i] = SA[i * sa_intv], sa[0] = -1) for bwt_sa."""

    def __init__(self, path: str | None = None, sa=None, sa_intv: int = 32, seq_len: int = 0):
        lib = load()
        if path is not None:
            self._h = lib.orc_sa_load(path.encode())
            if not self._h:
                raise IOError(path)
            self._keep = None
        else:
            a = np.ascontiguousarray(sa, dtype=np.uint64)
            self._keep = a
            self._h = lib.orc_sa_wrap(a.ctypes.data, a.size, int(sa_intv), int(seq_len))

    def lookup(self, index: OracleIndex, k) -> np.ndarray:
        """bwt_sa(bwt, k) for every k (software/bwt.c:104-114)."""
        k = np.ascontiguousarray(k, dtype=np.uint64)
        out = np.zeros(max(k.size, 1), dtype=np.uint64)
        if k.size:
            load().orc_sa_batch(index._h, self._h, k.ctypes.data, k.size, out.ctypes.data, min(8, os.cpu_count() or 1))
        return out[:k.size]

    def close(self):
        if self._h:
            load().orc_sa_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def sa_queries(lists_per_read, min_seed_len: int = 19, max_occ: int = 500):
    """The bwt_sa arguments mem_insert_seed() generates from smem_next2's lists
    (software/bwamem.c:462-474): for every interval with seed length >=
    min_seed_len and x2 <= max_occ, x0 + j for j < x2.  Returns (per-read
    counts, concatenated k)."""
    counts, ks = [], []
    for lists in lists_per_read:
        n = 0
        for a in lists:
            if a.shape[0] == 0:
                continue
            x0, x2, info = a[:, 0], a[:, 2], a[:, 3]
            slen = (info & 0xFFFFFFFF).astype(np.int64) - (info >> 32).astype(np.int64)
            for i in np.nonzero((slen >= min_seed_len) & (x2 <= max_occ))[0]:
                ks.append(x0[i] + np.arange(int(x2[i]), dtype=np.uint64))
                n += int(x2[i])
        counts.append(n)
    k = np.concatenate(ks).astype(np.uint64) if ks else np.zeros(0, np.uint64)
    return np.array(counts, dtype=np.int64), k


def ref_sa(bwt: str, sa: str, smgo: str, out: str, min_seed_len: int = 19, max_occ: int = 500) -> None:
    """bwt_sa of every seed occurrence of an SMGO stream, by the compiled reference."""
    subprocess.run([REF, "sa", bwt, sa, smgo, out, str(min_seed_len), str(max_occ)], check=True)


def _opt(min_seed_len=19, split_factor=1.5, split_width=10, start_width=1) -> OptT:
    return OptT(min_seed_len, split_factor, split_width, start_width)


def seed(index: OracleIndex, codes: np.ndarray, offs: np.ndarray, threads: int = 1, **opt):
    """Run the restated seeding loop. Returns (smgo_bytes, per_read dict, stats dict)."""
    lib = load()
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    n = offs.size - 1
    n_intv = np.zeros(max(n, 1), dtype=np.uint32)
    n_calls = np.zeros(max(n, 1), dtype=np.uint32)
    nbytes = np.zeros(max(n, 1), dtype=np.uint64)
    out = C.POINTER(C.c_uint8)()
    out_len = C.c_uint64()
    st = Stats()
    o = _opt(**opt)
    rc = lib.orc_seed(index._h, n, codes.ctypes.data, offs.ctypes.data, C.byref(o), threads, C.byref(out),
                      C.byref(out_len), n_intv.ctypes.data, n_calls.ctypes.data, nbytes.ctypes.data, C.byref(st))
    if rc != 0:
        raise RuntimeError("orc_seed failed")
    data = C.string_at(out, out_len.value)
    lib.orc_free(out)
    return data, {"n_intv": n_intv[:n], "n_calls": n_calls[:n], "bytes": nbytes[:n]}, st.as_dict()


def seed_trace(index: OracleIndex, codes: np.ndarray, offs: np.ndarray, **opt):
    """Occ64 bucket index of every load the GPU seeding kernel makes, in
    extend order (bit 31: an extend's second bucket), and the per-read
    offsets into it (orc_seed_trace; for tools/replay_ceiling.py)."""
    lib = load()
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    n = offs.size - 1
    o = _opt(**opt)
    roff = np.zeros(n + 1, dtype=np.uint64)
    cap = max(1, int(3000 * n))
    while True:
        buf = np.zeros(cap, dtype=np.uint32)
        tot = lib.orc_seed_trace(index._h, n, codes.ctypes.data, offs.ctypes.data, C.byref(o), buf.ctypes.data,
                                 cap, roff.ctypes.data)
        if tot < 0:
            raise RuntimeError("orc_seed_trace failed")
        if tot <= cap:
            return buf[:tot], roff
        cap = int(tot)


def seed_stats(index: OracleIndex, codes, offs, threads: int = 1, **opt):
    """Counters only (no stream materialised)."""
    _, per, st = seed(index, codes, offs, threads, **opt)
    return per, st


def seed_timed(index: OracleIndex, codes, offs, threads: int = 1, **opt):
    lib = load()
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    st = Stats()
    o = _opt(**opt)
    t = lib.orc_seed_timed(index._h, offs.size - 1, codes.ctypes.data, offs.ctypes.data, C.byref(o), threads,
                           C.byref(st))
    return float(t), st.as_dict()


def ref_available() -> bool:
    return os.path.exists(REF)


def ref_index(fasta: str, prefix: str) -> None:
    """bwa index -a is via the compiled reference."""
    subprocess.run([REF, "index", fasta, prefix], check=True, capture_output=True)


def ref_smem(bwt: str, smrd: str, out: str, min_seed_len=19, split_factor=1.5, split_width=10, start_width=1) -> None:
    subprocess.run([REF, "smem", bwt, smrd, out, str(min_seed_len), str(split_factor), str(split_width),
                    str(start_width)], check=True)


def ref_bench(bwt: str, smrd: str, threads: int, max_reads: int, min_seed_len=19, split_factor=1.5, split_width=10,
              start_width=1) -> dict:
    p = subprocess.run([REF, "bench", bwt, smrd, str(threads), str(max_reads), str(min_seed_len), str(split_factor),
                        str(split_width), str(start_width)], check=True, capture_output=True, text=True)
    kv = dict(tok.split("=") for tok in p.stdout.split())
    return {k: float(v) for k, v in kv.items()}


SEED_DT = np.dtype([("rbeg", "<i8"), ("qbeg", "<i4"), ("len", "<i4")])  # mem_seed_t


def chain_seeds(lists_per_read, positions_per_read, min_seed_len: int = 19, max_occ: int = 10000):
    """The seed sequence mem_insert_seed generates (software/bwamem.c:462-474):
    for every interval with seed length >= min_seed_len and x2 <= max_occ, in
    order, one (rbeg = bwt_sa(x0 + j), qbeg, len) per occurrence j < x2.
    positions_per_read are those bwt_sa values (an SMSA stream's). Returns
    (seeds SEED_DT array, seed_off[n_reads + 1])."""
    parts, counts = [], []
    for lists, pos in zip(lists_per_read, positions_per_read):
        q, l = [], []
        for a in lists:
            if a.shape[0] == 0:
                continue
            x2, info = a[:, 2], a[:, 3]
            beg = (info >> 32).astype(np.int64)
            slen = (info & 0xFFFFFFFF).astype(np.int64) - beg
            keep = (slen >= min_seed_len) & (x2 <= max_occ)
            rep = np.where(keep, x2, 0).astype(np.int64)
            q.append(np.repeat(beg, rep))
            l.append(np.repeat(slen, rep))
        qb = np.concatenate(q) if q else np.zeros(0, np.int64)
        if qb.size != len(pos):
            raise ValueError("positions do not match the lists")
        s = np.zeros(qb.size, dtype=SEED_DT)
        s["rbeg"] = np.asarray(pos, dtype=np.uint64).view(np.int64)
        s["qbeg"] = qb
        s["len"] = np.concatenate(l) if l else 0
        parts.append(s)
        counts.append(qb.size)
    seeds = np.concatenate(parts) if parts else np.zeros(0, SEED_DT)
    off = np.concatenate([[0], np.cumsum(counts, dtype=np.uint64)]).astype(np.uint64)
    return seeds, off


def chain(seeds, seed_off, l_pac: int, w=100, max_chain_gap=10000, min_seed_len=19, mask_level=0.5,
          drop_ratio=0.5, filter=1, threads: int = 1) -> bytes:
    """mem_chain (+ mem_chain_flt when filter) of every read: SMCH bytes."""
    lib = load()
    seeds = np.ascontiguousarray(seeds, dtype=SEED_DT)
    seed_off = np.ascontiguousarray(seed_off, dtype=np.uint64)
    o = ChainOptT(w, max_chain_gap, min_seed_len, mask_level, drop_ratio, int(filter))
    out = C.POINTER(C.c_uint8)()
    out_len = C.c_uint64()
    sp = seeds.ctypes.data if seeds.size else None
    rc = lib.orc_chain(seed_off.size - 1, sp, seed_off.ctypes.data, int(l_pac), C.byref(o), threads, C.byref(out),
                       C.byref(out_len))
    if rc != 0:
        raise RuntimeError("orc_chain failed")
    data = C.string_at(out, out_len.value)
    lib.orc_free(out)
    return data


# ---- SW extension (ksw_oracle.c) -------------------------------------------
def ksw_opt(batch) -> KswOptT:
    o = KswOptT()
    for i, v in enumerate(np.asarray(batch.mat, dtype=np.int8)):
        o.mat[i] = int(v)
    o.o_del, o.e_del, o.o_ins, o.e_ins = batch.o_del, batch.e_del, batch.o_ins, batch.e_ins
    return o


def ksw(batch) -> np.ndarray:
    """The restated ksw_extend2 on every task of a synth.KswBatch."""
    from smemgpu import synth
    lib = load()
    tasks = np.ascontiguousarray(batch.tasks, dtype=synth.KSW_TASK)
    q = np.ascontiguousarray(batch.q, dtype=np.uint8)
    t = np.ascontiguousarray(batch.t, dtype=np.uint8)
    out = np.zeros(max(tasks.size, 1), dtype=synth.KSW_RESULT)
    o = ksw_opt(batch)
    rc = lib.orc_ksw_batch(tasks.size, tasks.ctypes.data, q.ctypes.data, t.ctypes.data, C.byref(o), out.ctypes.data)
    if rc != 0:
        raise RuntimeError("orc_ksw_batch failed")
    return out[:tasks.size]


def ksw_align2(batch) -> np.ndarray:
    """The restatement's ksw_align2 (aln_oracle.c sw_align) of every task of a
    synth.KswBatch of KSWA_TASK problems, as synth.KSWA_RESULT."""
    from smemgpu import synth
    lib = load()
    mat = np.ascontiguousarray(batch.mat, dtype=np.int8)
    out = np.zeros(batch.tasks.size, dtype=synth.KSWA_RESULT)
    r = (C.c_int32 * 7)()
    for i, t in enumerate(batch.tasks):
        q = np.ascontiguousarray(batch.q[int(t["q_off"]):int(t["q_off"]) + int(t["qlen"])])
        tg = np.ascontiguousarray(batch.t[int(t["t_off"]):int(t["t_off"]) + int(t["tlen"])])
        lib.orc_ksw_align2(int(t["qlen"]), q.ctypes.data, int(t["tlen"]), tg.ctypes.data if tg.size else None,
                           mat.ctypes.data, batch.o_del, batch.e_del, batch.o_ins, batch.e_ins, int(t["xtra"]), r)
        out[i] = tuple(r)
    return out


def ref_aln_time(bwt: str, sa: str, pac: str, smrd: str, min_seed_len=19, w=100) -> dict:
    """The reference's mem_chain + mem_chain_flt + chain2aln loop over a read
    file (ref_harness aln), returning the time of the chain2aln loop alone."""
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        p = subprocess.run([REF, "aln", bwt, sa, pac, smrd, os.path.join(d, "o.smrg"), str(min_seed_len), "1.5", "10",
                            "1", "10000", str(w), "10000", "0.5", "0.5"], check=True, capture_output=True, text=True)
    line = [l for l in p.stderr.split("\n") if l.startswith("chain2aln_seconds=")][-1]
    return {k: float(v) for k, v in (t.split("=") for t in line.split())}


def ref_kswa(smat: str, out: str) -> None:
    subprocess.run([REF, "kswa", smat, out], check=True, capture_output=True)


def ref_ksw(smkt: str, out: str) -> None:
    """The compiled reference's own ksw_extend2 on every task of an SMKT file."""
    subprocess.run([REF, "ksw", smkt, out], check=True)


# ---- chains -> regions (aln_oracle.c) --------------------------------------
class AlnOptT(C.Structure):
    """orc_aln_opt_t (= smem_aln_opt_t)"""
    _fields_ = [("mat", C.c_int8 * 25), ("pad", C.c_int8 * 3), ("o_del", C.c_int32), ("e_del", C.c_int32),
                ("o_ins", C.c_int32), ("e_ins", C.c_int32), ("a", C.c_int32), ("w", C.c_int32), ("zdrop", C.c_int32),
                ("pen_clip5", C.c_int32), ("pen_clip3", C.c_int32), ("min_seed_len", C.c_int32)]


def aln_opt(w=100, min_seed_len=19, a=1, b=4, o_del=6, e_del=1, o_ins=6, e_ins=1, zdrop=100, pen_clip5=5,
            pen_clip3=5) -> AlnOptT:
    """mem_opt_init's scoring (software/bwamem.c:47-70), bwa_fill_scmat (software/bwa.c:84-93)"""
    o = AlnOptT()
    for i in range(4):
        for j in range(4):
            o.mat[i * 5 + j] = a if i == j else -b
        o.mat[i * 5 + 4] = -1
    for j in range(5):
        o.mat[20 + j] = -1
    o.o_del, o.e_del, o.o_ins, o.e_ins, o.a, o.w, o.zdrop = o_del, e_del, o_ins, e_ins, a, w, zdrop
    o.pen_clip5, o.pen_clip3, o.min_seed_len = pen_clip5, pen_clip3, min_seed_len
    return o


def dp_cells(reset: bool = True) -> tuple:
    """(ksw_extend2 in-band cells, ksw_align2 query x target cells) the
    restatement computed on this thread since the last reset: the DP stages'
    algorithmic work (ksw_oracle.c orc_cells)."""
    out = (C.c_uint64 * 2)()
    load().orc_cells(out, 1 if reset else 0)
    return int(out[0]), int(out[1])


def ext_shapes(reset: bool = True) -> list:
    """[(calls, in-band cells)] of the restatement's chain2aln extensions by
    qlen bucket (<= 16, 32, 64, 128, 256, longer) on this thread."""
    out = (C.c_uint64 * 12)()
    load().orc_ext_shapes(out, 1 if reset else 0)
    return [(int(out[2 * b]), int(out[2 * b + 1])) for b in range(6)]


def seed_uses(reset: bool = True) -> dict:
    """Which seeds the restatement's chain2aln extended on this thread: the
    chain's first seed in the order (longest) or another, first seeds skipped
    as contained, and the seeds of the chains it ran on."""
    out = (C.c_uint64 * 4)()
    load().orc_seed_uses(out, 1 if reset else 0)
    return dict(first_extended=int(out[0]), other_extended=int(out[1]), first_skipped=int(out[2]),
                seeds=int(out[3]))


def aln(pac, l_pac: int, codes, offs, chains, chain_off, seeds, opt: AlnOptT):
    """The restated mem_chain2aln_short / mem_chain2aln loop over every read's
    chains: (regions as golden_data.ALNREG_DT, reg_off[n_reads + 1])."""
    from tests.golden_data import ALNREG_DT
    lib = load()
    pac = np.ascontiguousarray(pac, dtype=np.uint8)
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    chain_off = np.ascontiguousarray(chain_off, dtype=np.uint64)
    chains = np.ascontiguousarray(chains)
    seeds = np.ascontiguousarray(seeds)
    n = offs.size - 1
    reg_off = np.zeros(n + 1, dtype=np.uint64)
    p = C.c_void_p()
    rc = lib.orc_aln_batch(C.byref(opt), l_pac, pac.ctypes.data, n, codes.ctypes.data, offs.ctypes.data,
                           chains.ctypes.data, chain_off.ctypes.data, seeds.ctypes.data, C.byref(p),
                           reg_off.ctypes.data)
    if rc != 0:
        raise RuntimeError("orc_aln_batch failed")
    k = int(reg_off[-1])
    out = np.frombuffer((C.c_uint8 * (k * 64)).from_address(p.value), dtype=ALNREG_DT).copy() if k else \
        np.zeros(0, dtype=ALNREG_DT)
    lib.orc_free(p)
    return out, reg_off

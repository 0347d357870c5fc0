"""ctypes binding of libsmemgpu.so (include/smem_gpu.h).

The library is built in-tree by `make -C bwa-mem-harp2_amd` (or
__graft_entry__.build()).  Loading fails loudly if it is missing: there is no
Python or CPU fallback for the seeding path.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("SMEMGPU_LIB") or os.path.join(PKG_DIR, "lib", "libsmemgpu.so")  # override: A/B builds

SMEM_OK = 0
ERRORS = {-1: "SMEM_E_ARG", -2: "SMEM_E_NOMEM", -3: "SMEM_E_IO", -4: "SMEM_E_DEVICE",
          -5: "SMEM_E_INTERNAL", -6: "SMEM_E_CAPACITY"}

# every symbol include/smem_gpu.h declares
EXPORTED = [
    "smem_opt_default", "smem_bwt_build", "smem_bwt_build_gpu", "smem_bwt_read", "smem_bwt_write", "smem_index_free",
    "smem_gpu_device_count", "smem_gpu_init", "smem_gpu_shutdown", "smem_gpu_collect",
    "smem_batch_create", "smem_batch_destroy", "smem_batch_set_reads", "smem_batch_set_reads_packed",
    "smem_batch_run", "smem_batch_fetch", "smem_batch_read", "smem_batch_results", "smem_batch_stats",
    "smem_gpu_set_lanes_per_cu", "smem_gpu_set_intv_cap", "smem_gpu_set_kernel_variant", "smem_gpu_get_kernel_variant", "smem_gpu_grid_reads", "smem_gpu_set_kmer_table", "smem_batch_debug", "smem_strerror",
    "smem_gpu_build_id",
    "smem_bwt_build_sa", "smem_bwt_build_gpu_sa", "smem_sa_read", "smem_sa_write", "smem_sa_free", "smem_gpu_load_sa",
    "smem_batch_sa", "smem_batch_sa_results",
    "smem_chain_opt_default", "smem_batch_chain", "smem_batch_chain_results", "smem_bwt_build_gpu_large",
    "smem_ksw_opt_default", "smem_ksw_extend", "smem_aln_opt_default", "smem_chain2aln",
    "smem_gpu_seed_stream", "smem_batch_results_packed",
    "smem_gpu_load_pac", "smem_batch_chain2aln", "smem_batch_aln_results", "smem_ksw_align2",
    "smem_gpu_init_devices", "smem_gpu_parse_devices", "smem_gpu_collect_ex", "smem_batch_fetch_mask",
    "smem_gpu_reserve_slots", "smem_gpu_set_max_active", "smem_gpu_get_max_active", "smem_gpu_kernel_id", "smem_gpu_fault",
    "smem_batch_memory", "smem_gpu_memory", "smem_gpu_init_devices_async", "smem_gpu_wait_ready",
    "smem_gpu_open_async", "smem_gpu_load_sa_async", "smem_gpu_load_pac_async",
]

# smem_batch_fetch_mask bits (include/smem_gpu.h)
FETCH_INTV, FETCH_SA, FETCH_CHAINS, FETCH_REGS, FETCH_ALL = 1, 2, 4, 8, 15
COLLECT_NO_FETCH = 1


def source_hash() -> str:
    """The content hash bwa-mem-harp2_amd/Makefile compiles into the library
    (SRC_HASH): sha256 of csrc/*.{hip,cpp,c,h}, include/*.h and the Makefile
    (its compiler flags), concatenated in path order, first 16 hex digits."""
    import glob
    import hashlib
    inc = os.path.join(os.path.dirname(PKG_DIR), "include")
    files = sorted(glob.glob(os.path.join(PKG_DIR, "csrc", "*.hip")) + glob.glob(os.path.join(PKG_DIR, "csrc", "*.cpp"))
                   + glob.glob(os.path.join(PKG_DIR, "csrc", "*.c")) + glob.glob(os.path.join(PKG_DIR, "csrc", "*.h"))
                   + glob.glob(os.path.join(inc, "*.h")) + [os.path.join(PKG_DIR, "Makefile")])
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_id() -> str:
    """The source hash the loaded libsmemgpu.so was built from."""
    return load().smem_gpu_build_id().decode()


def kernel_id() -> str:
    """Hash of the loaded library's seeding-kernel sources and compile flags only
    (bwa-mem-harp2_amd/Makefile KERNEL_HASH): seed_kernel counters recorded on
    another build of the runtime still describe it when this id matches."""
    return load().smem_gpu_kernel_id().decode()


class SmemError(RuntimeError):
    pass


class Intv(C.Structure):
    _fields_ = [("x", C.c_uint64 * 3), ("info", C.c_uint64)]


class IndexT(C.Structure):
    _fields_ = [("primary", C.c_uint64), ("L2", C.c_uint64 * 5), ("seq_len", C.c_uint64),
                ("bwt_size", C.c_uint64), ("bwt", C.POINTER(C.c_uint32)), ("owns", C.c_int)]


class SaT(C.Structure):
    _fields_ = [("primary", C.c_uint64), ("L2", C.c_uint64 * 5), ("seq_len", C.c_uint64), ("sa_intv", C.c_uint64),
                ("n_sa", C.c_uint64), ("sa", C.POINTER(C.c_uint64)), ("owns", C.c_int)]


class OptT(C.Structure):
    _fields_ = [("min_seed_len", C.c_int), ("split_factor", C.c_float), ("split_width", C.c_int),
                ("start_width", C.c_int)]


class BatchStats(C.Structure):
    _fields_ = [("kernel_ms", C.c_double), ("compact_ms", C.c_double), ("n_intv", C.c_uint64),
                ("n_calls", C.c_uint64), ("n_overflow", C.c_uint32), ("grid", C.c_int), ("block", C.c_int),
                ("sa_ms", C.c_double), ("n_occ", C.c_uint64), ("chain_ms", C.c_double), ("n_chains", C.c_uint64),
                ("aln_ms", C.c_double), ("n_regs", C.c_uint64), ("t_start", C.c_uint64), ("t_end", C.c_uint64)]


class StreamStats(C.Structure):
    """smem_stream_stats_t"""
    _fields_ = [("wall_s", C.c_double), ("n_reads", C.c_uint64), ("n_chunks", C.c_uint64), ("n_intv", C.c_uint64),
                ("h2d_bytes", C.c_uint64), ("d2h_bytes", C.c_uint64), ("workers", C.c_int), ("stage_s", C.c_double),
                ("run_s", C.c_double), ("fetch_s", C.c_double)]


# int (*smem_chunk_fn)(void *ctx, int64_t chunk, int64_t first_read, int n_reads, const smem_batch_t *b)
CHUNK_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64, C.c_int64, C.c_int, C.c_void_p)


class KswOptT(C.Structure):
    """smem_ksw_opt_t"""
    _fields_ = [("mat", C.c_int8 * 25), ("pad", C.c_int8 * 3), ("o_del", C.c_int32), ("e_del", C.c_int32),
                ("o_ins", C.c_int32), ("e_ins", C.c_int32)]


class ChainOptT(C.Structure):
    _fields_ = [("w", C.c_int), ("max_chain_gap", C.c_int), ("mask_level", C.c_float),
                ("chain_drop_ratio", C.c_float), ("filter", C.c_int)]


class AlnOptT(C.Structure):
    """smem_aln_opt_t: the mem_opt_t fields mem_chain2aln reads"""
    _fields_ = [("mat", C.c_int8 * 25), ("pad", C.c_int8 * 3), ("o_del", C.c_int32), ("e_del", C.c_int32),
                ("o_ins", C.c_int32), ("e_ins", C.c_int32), ("a", C.c_int32), ("w", C.c_int32), ("zdrop", C.c_int32),
                ("pen_clip5", C.c_int32), ("pen_clip3", C.c_int32), ("min_seed_len", C.c_int32)]


def aln_opt(**kw) -> AlnOptT:
    """smem_aln_opt_default (mem_opt_init's scoring, software/bwamem.c:47-70)
    with the named fields overridden (e.g. min_seed_len=19, w=100)."""
    o = AlnOptT()
    load().smem_aln_opt_default(C.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


SEED_DT = np.dtype([("rbeg", "<i8"), ("qbeg", "<i4"), ("len", "<i4")])          # smem_seed_t = mem_seed_t
CHAIN_DT = np.dtype([("pos", "<i8"), ("seed_off", "<u8"), ("n", "<i4"), ("pad", "<i4")])  # smem_chain_t


_lib = None


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SmemError(f"{LIB_PATH} is missing: build it with `make -C {PKG_DIR}` (no fallback exists)")
    lib = C.CDLL(LIB_PATH)
    P = C.POINTER
    lib.smem_opt_default.argtypes = [P(OptT)]
    lib.smem_opt_default.restype = None
    lib.smem_bwt_build.argtypes = [C.c_void_p, C.c_uint64, P(IndexT)]
    lib.smem_bwt_build_gpu.argtypes = [C.c_int, C.c_void_p, C.c_uint64, P(IndexT)]
    lib.smem_bwt_read.argtypes = [C.c_char_p, P(IndexT)]
    lib.smem_bwt_write.argtypes = [C.c_char_p, P(IndexT)]
    lib.smem_index_free.argtypes = [P(IndexT)]
    lib.smem_index_free.restype = None
    lib.smem_bwt_build_sa.argtypes = [C.c_void_p, C.c_uint64, C.c_int, P(IndexT), P(SaT)]
    lib.smem_bwt_build_gpu_sa.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_int, P(IndexT), P(SaT)]
    lib.smem_bwt_build_gpu_large.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_int, P(IndexT), P(SaT)]
    lib.smem_sa_read.argtypes = [C.c_char_p, P(SaT)]
    lib.smem_sa_write.argtypes = [C.c_char_p, P(SaT)]
    lib.smem_sa_free.argtypes = [P(SaT)]
    lib.smem_sa_free.restype = None
    lib.smem_gpu_load_sa.argtypes = [C.c_void_p, P(SaT)]
    lib.smem_batch_sa.argtypes = [C.c_void_p, C.c_int, C.c_int]
    lib.smem_batch_sa_results.argtypes = [C.c_void_p, P(P(C.c_uint64)), P(P(C.c_uint64)), P(C.c_uint64)]
    lib.smem_ksw_opt_default.argtypes = [P(KswOptT)]
    lib.smem_ksw_opt_default.restype = None
    lib.smem_ksw_extend.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                    P(KswOptT), C.c_void_p, P(C.c_double)]
    lib.smem_aln_opt_default.argtypes = [C.c_void_p]
    lib.smem_aln_opt_default.restype = None
    lib.smem_chain2aln.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.c_uint64, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                                   P(C.c_double)]
    lib.smem_chain_opt_default.argtypes = [P(ChainOptT)]
    lib.smem_chain_opt_default.restype = None
    lib.smem_batch_chain.argtypes = [C.c_void_p, C.c_int64, P(ChainOptT)]
    lib.smem_batch_chain_results.argtypes = [C.c_void_p, P(C.c_void_p), P(P(C.c_uint64)), P(C.c_void_p),
                                             P(C.c_uint64), P(C.c_uint64)]
    lib.smem_gpu_device_count.argtypes = []
    lib.smem_gpu_init.argtypes = [P(C.c_void_p), C.c_int, C.c_void_p, C.c_uint64, C.c_uint64, P(C.c_uint64)]
    lib.smem_gpu_shutdown.argtypes = [C.c_void_p]
    lib.smem_gpu_shutdown.restype = None
    lib.smem_gpu_collect.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, P(OptT), P(C.c_void_p)]
    lib.smem_gpu_collect_ex.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, P(OptT), C.c_int,
                                        P(C.c_void_p)]
    lib.smem_gpu_init_devices.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64,
                                          P(C.c_uint64), C.c_void_p, C.c_void_p, C.c_int64]
    lib.smem_gpu_parse_devices.argtypes = [C.c_char_p, C.c_void_p, C.c_int]
    lib.smem_batch_fetch_mask.argtypes = [C.c_void_p, C.c_int]
    lib.smem_gpu_seed_stream.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, P(OptT), C.c_int, C.c_int,
                                         C.c_int, C.c_void_p, C.c_void_p, P(StreamStats)]
    lib.smem_ksw_align2.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                    P(KswOptT), C.c_void_p, P(C.c_double)]
    lib.smem_gpu_load_pac.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    lib.smem_batch_chain2aln.argtypes = [C.c_void_p, C.c_void_p]
    lib.smem_batch_aln_results.argtypes = [C.c_void_p, P(C.c_void_p), P(P(C.c_uint64)), P(C.c_uint64)]
    lib.smem_batch_results_packed.argtypes = [C.c_void_p, P(C.c_void_p), P(P(C.c_uint64)), P(P(C.c_uint32)),
                                              P(P(C.c_uint64))]
    lib.smem_batch_create.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.c_int, P(C.c_void_p)]
    lib.smem_batch_destroy.argtypes = [C.c_void_p]
    lib.smem_batch_destroy.restype = None
    lib.smem_batch_set_reads.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    lib.smem_batch_set_reads_packed.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    lib.smem_batch_run.argtypes = [C.c_void_p, P(OptT)]
    lib.smem_batch_fetch.argtypes = [C.c_void_p]
    lib.smem_batch_read.argtypes = [C.c_void_p, C.c_int, P(P(Intv)), P(C.c_int), P(P(C.c_uint32)), P(C.c_int)]
    lib.smem_batch_results.argtypes = [C.c_void_p, P(P(Intv)), P(P(C.c_uint64)), P(P(C.c_uint32)), P(P(C.c_uint64))]
    lib.smem_batch_stats.argtypes = [C.c_void_p, P(BatchStats)]
    lib.smem_gpu_set_lanes_per_cu.argtypes = [C.c_void_p, C.c_int]
    lib.smem_gpu_set_intv_cap.argtypes = [C.c_void_p, C.c_int]
    lib.smem_gpu_set_kernel_variant.argtypes = [C.c_void_p, C.c_int]
    lib.smem_gpu_get_kernel_variant.argtypes = [C.c_void_p]
    lib.smem_gpu_get_kernel_variant.restype = C.c_int
    lib.smem_gpu_grid_reads.argtypes = [C.c_void_p]
    lib.smem_gpu_grid_reads.restype = C.c_int
    lib.smem_gpu_set_kmer_table.argtypes = [C.c_void_p, C.c_int]
    if hasattr(lib, "smem_batch_debug"):  # absent from older A/B builds
        lib.smem_batch_debug.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
    lib.smem_strerror.argtypes = [C.c_int]
    lib.smem_strerror.restype = C.c_char_p
    lib.smem_gpu_build_id.argtypes = []
    lib.smem_gpu_build_id.restype = C.c_char_p
    lib.smem_gpu_kernel_id.argtypes = []
    lib.smem_gpu_kernel_id.restype = C.c_char_p
    lib.smem_gpu_reserve_slots.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int]
    lib.smem_gpu_set_max_active.argtypes = [C.c_void_p, C.c_int]
    lib.smem_gpu_get_max_active.argtypes = [C.c_void_p]
    lib.smem_gpu_fault.argtypes = [C.c_void_p, C.c_char_p, C.c_int]
    lib.smem_gpu_init_devices_async.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64,
                                                P(C.c_uint64), C.c_void_p, C.c_void_p, C.c_int64]
    lib.smem_gpu_wait_ready.argtypes = [C.c_void_p]
    lib.smem_batch_memory.argtypes = [C.c_void_p, P(C.c_uint64), P(C.c_uint64)]
    lib.smem_gpu_memory.argtypes = [C.c_void_p, P(C.c_uint64), P(C.c_uint64), P(C.c_uint64), P(C.c_int)]
    _lib = lib
    return lib


def _check(rc: int, what: str) -> None:
    if rc != SMEM_OK:
        msg = load().smem_strerror(rc).decode(errors="replace")
        raise SmemError(f"{what} failed: {ERRORS.get(rc, rc)}: {msg}")


@dataclass
class Options:
    """mem_opt_t fields of the seeding loop (defaults: software/bwamem.c:58-65)."""
    min_seed_len: int = 19
    split_factor: float = 1.5
    split_width: int = 10
    start_width: int = 1

    def c(self) -> OptT:
        return OptT(self.min_seed_len, self.split_factor, self.split_width, self.start_width)


class Index:
    """BWA .bwt FM-index in host memory (owned by the library)."""

    def __init__(self, raw: IndexT):
        self._raw = raw

    @classmethod
    def build(cls, fwd_codes: np.ndarray) -> "Index":
        fwd = np.ascontiguousarray(fwd_codes, dtype=np.uint8)
        raw = IndexT()
        _check(load().smem_bwt_build(fwd.ctypes.data, fwd.size, C.byref(raw)), "smem_bwt_build")
        return cls(raw)

    @classmethod
    def build_gpu(cls, fwd_codes: np.ndarray, device: int = 0, large: bool = False) -> "Index":
        """Same bytes as build(), constructed on a HIP device (prefix doubling;
        large=True forces the bucketed 64-bit builder used past 2^32 symbols)."""
        fwd = np.ascontiguousarray(fwd_codes, dtype=np.uint8)
        raw = IndexT()
        if large:
            _check(load().smem_bwt_build_gpu_large(device, fwd.ctypes.data, fwd.size, 0, C.byref(raw), None),
                   "smem_bwt_build_gpu_large")
        else:
            _check(load().smem_bwt_build_gpu(device, fwd.ctypes.data, fwd.size, C.byref(raw)), "smem_bwt_build_gpu")
        return cls(raw)

    @classmethod
    def build_sa(cls, fwd_codes: np.ndarray, sa_intv: int = 32, gpu: bool = False, device: int = 0,
                 large: bool = False):
        """(Index, SA): the .bwt and the sampled SA bwa index writes beside it."""
        fwd = np.ascontiguousarray(fwd_codes, dtype=np.uint8)
        raw, sraw = IndexT(), SaT()
        if gpu and large:
            _check(load().smem_bwt_build_gpu_large(device, fwd.ctypes.data, fwd.size, sa_intv, C.byref(raw),
                                                   C.byref(sraw)), "smem_bwt_build_gpu_large")
        elif gpu:
            _check(load().smem_bwt_build_gpu_sa(device, fwd.ctypes.data, fwd.size, sa_intv, C.byref(raw), C.byref(sraw)),
                   "smem_bwt_build_gpu_sa")
        else:
            _check(load().smem_bwt_build_sa(fwd.ctypes.data, fwd.size, sa_intv, C.byref(raw), C.byref(sraw)),
                   "smem_bwt_build_sa")
        return cls(raw), SA(sraw)

    @classmethod
    def read(cls, path: str) -> "Index":
        raw = IndexT()
        _check(load().smem_bwt_read(path.encode(), C.byref(raw)), f"smem_bwt_read({path})")
        return cls(raw)

    def write(self, path: str) -> None:
        _check(load().smem_bwt_write(path.encode(), C.byref(self._raw)), f"smem_bwt_write({path})")

    @property
    def primary(self) -> int:
        return int(self._raw.primary)

    @property
    def L2(self) -> np.ndarray:
        return np.array(list(self._raw.L2), dtype=np.uint64)

    @property
    def seq_len(self) -> int:
        return int(self._raw.seq_len)

    @property
    def words(self) -> np.ndarray:
        """uint32 view (no copy) of the interleaved BWT + Occ words."""
        n = int(self._raw.bwt_size)
        return np.ctypeslib.as_array(self._raw.bwt, shape=(n,))

    def close(self) -> None:
        if self._raw.bwt:
            load().smem_index_free(C.byref(self._raw))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SA:
    """Sampled suffix array (.sa) in host memory (owned by the library)."""

    def __init__(self, raw: SaT):
        self._raw = raw

    @classmethod
    def read(cls, path: str) -> "SA":
        raw = SaT()
        _check(load().smem_sa_read(path.encode(), C.byref(raw)), f"smem_sa_read({path})")
        return cls(raw)

    def write(self, path: str) -> None:
        _check(load().smem_sa_write(path.encode(), C.byref(self._raw)), f"smem_sa_write({path})")

    @property
    def sa_intv(self) -> int:
        return int(self._raw.sa_intv)

    @property
    def seq_len(self) -> int:
        return int(self._raw.seq_len)

    @property
    def samples(self) -> np.ndarray:
        """uint64 view (no copy) of sa[0 .. n_sa-1]; sa[0] = 2^64-1."""
        return np.ctypeslib.as_array(self._raw.sa, shape=(int(self._raw.n_sa),))

    def close(self) -> None:
        if self._raw.sa:
            load().smem_sa_free(C.byref(self._raw))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def device_count() -> int:
    return int(load().smem_gpu_device_count())


@dataclass
class Results:
    intv: np.ndarray      # (N, 4) uint64: x0, x1, x2, info
    intv_off: np.ndarray  # (n_reads + 1,) uint64
    call_n: np.ndarray    # (n_lists,) uint32
    call_off: np.ndarray  # (n_reads + 1,) uint64
    occ_off: np.ndarray | None = None  # (N + 1,) uint64, when Batch.sa() ran
    sa_pos: np.ndarray | None = None   # (n_occ,) uint64 bwt_sa positions
    chains: np.ndarray | None = None   # CHAIN_DT, when Batch.chain() ran
    chain_off: np.ndarray | None = None  # (n_reads + 1,) uint64
    seeds: np.ndarray | None = None    # SEED_DT, each chain's seeds contiguous
    regs: np.ndarray | None = None     # raw 64-byte smem_alnreg_t records, when Batch.chain2aln() ran
    reg_off: np.ndarray | None = None  # (n_reads + 1,) uint64

    def read_chains(self, i: int) -> list:
        """read i's chains as [(pos, seeds)], in mem_chain(+flt) order."""
        out = []
        for c in self.chains[int(self.chain_off[i]):int(self.chain_off[i + 1])]:
            o = int(c["seed_off"])
            out.append((int(c["pos"]), self.seeds[o:o + int(c["n"])]))
        return out

    def to_smch(self) -> bytes:
        from . import synth
        return synth.write_smch([self.read_chains(i) for i in range(self.chain_off.size - 1)])

    def read_sa(self, i: int) -> np.ndarray:
        """bwt_sa positions of read i's seed occurrences, in interval order."""
        a, b = int(self.intv_off[i]), int(self.intv_off[i + 1])
        return self.sa_pos[int(self.occ_off[a]):int(self.occ_off[b])]

    def to_smsa(self) -> bytes:
        from . import synth
        return synth.write_smsa([self.read_sa(i) for i in range(self.intv_off.size - 1)])

    def read_calls(self, i: int) -> list:
        """The lists smem_next2 returned for read i, in order."""
        iv = self.intv[self.intv_off[i]:self.intv_off[i + 1]]
        ns = self.call_n[self.call_off[i]:self.call_off[i + 1]]
        out, p = [], 0
        for n in ns:
            out.append(iv[p:p + int(n)])
            p += int(n)
        return out

    def to_smgo(self) -> bytes:
        import struct
        n = self.intv_off.size - 1
        parts = [b"SMGO0001", struct.pack("<Q", n)]
        for i in range(n):
            calls = self.read_calls(i)
            parts.append(struct.pack("<I", len(calls)))
            for arr in calls:
                parts.append(struct.pack("<I", arr.shape[0]))
                parts.append(np.ascontiguousarray(arr, dtype="<u8").tobytes())
        return b"".join(parts)


class Gpu:
    """One HIP device with the index resident in HBM (smem_gpu_init)."""

    def __init__(self, index: Index, device: int = 0, lanes_per_cu: int = 0, intv_cap: int = 0, variant: int = 0,
                 kmer_k: int = 0):
        lib = load()
        self._h = C.c_void_p()
        words = index.words
        L2 = (C.c_uint64 * 5)(*[int(v) for v in index.L2])
        _check(lib.smem_gpu_init(C.byref(self._h), device, words.ctypes.data, words.size, index.primary, L2),
               "smem_gpu_init")
        if lanes_per_cu:
            _check(lib.smem_gpu_set_lanes_per_cu(self._h, lanes_per_cu), "smem_gpu_set_lanes_per_cu")
        if intv_cap:
            _check(lib.smem_gpu_set_intv_cap(self._h, intv_cap), "smem_gpu_set_intv_cap")
        if kmer_k:
            self.set_kmer_table(kmer_k)
        if variant:
            _check(lib.smem_gpu_set_kernel_variant(self._h, variant), "smem_gpu_set_kernel_variant")
        self.device = device

    @classmethod
    def open_async(cls, index: Index, devices, sa: "SA" = None, pac=None, l_pac: int = 0) -> list:
        """smem_gpu_init_devices_async: one Gpu per entry of `devices`, whose
        uploads run in the background (index, sa and pac must outlive them:
        keep the objects alive until wait_ready() or close())."""
        lib = load()
        n = len(devices)
        hs = (C.c_void_p * n)()
        devs = (C.c_int * n)(*devices)
        words = index.words
        L2 = (C.c_uint64 * 5)(*[int(v) for v in index.L2])
        pac_p = np.ascontiguousarray(pac, dtype=np.uint8).ctypes.data if pac is not None else None
        _check(lib.smem_gpu_init_devices_async(hs, n, devs, words.ctypes.data, words.size, index.primary, L2,
                                               C.byref(sa._raw) if sa is not None else None, pac_p, int(l_pac)),
               "smem_gpu_init_devices_async")
        out = []
        for i in range(n):
            g = cls.__new__(cls)
            g._h = C.c_void_p(hs[i])
            g.device = devices[i]
            out.append(g)
        return out

    def wait_ready(self) -> None:
        _check(load().smem_gpu_wait_ready(self._h), "smem_gpu_wait_ready")

    def set_variant(self, variant: int) -> None:
        """Seeding-kernel variant (0 = default; see smem_gpu_set_kernel_variant)."""
        _check(load().smem_gpu_set_kernel_variant(self._h, variant), "smem_gpu_set_kernel_variant")

    @property
    def grid_reads(self) -> int:
        """Reads one seeding launch holds in flight (smem_gpu_grid_reads)."""
        return int(load().smem_gpu_grid_reads(self._h))

    @property
    def variant(self) -> int:
        """The seeding-kernel variant this handle runs (smem_gpu_get_kernel_variant)."""
        return int(load().smem_gpu_get_kernel_variant(self._h))

    def set_kmer_table(self, k: int) -> None:
        """Build (k = 1..15) or free (0) the device k-mer bi-interval table."""
        _check(load().smem_gpu_set_kmer_table(self._h, k), "smem_gpu_set_kmer_table")

    def load_sa(self, sa: "SA") -> None:
        _check(load().smem_gpu_load_sa(self._h, C.byref(sa._raw)), "smem_gpu_load_sa")

    def set_max_active(self, n: int) -> None:
        """Admission: at most n calls on the device at once (smem_gpu_set_max_active; 0 = default)."""
        _check(load().smem_gpu_set_max_active(self._h, n), "smem_gpu_set_max_active")

    def max_active(self) -> int:
        """The admission limit in force (smem_gpu_get_max_active)."""
        rc = load().smem_gpu_get_max_active(self._h)
        if rc < 0:
            _check(rc, "smem_gpu_get_max_active")
        return rc

    def memory(self) -> dict:
        """smem_gpu_memory: bytes of the resident index, of the kept batches (device / pinned)."""
        ix, d, h, nb = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_int()
        _check(load().smem_gpu_memory(self._h, C.byref(ix), C.byref(d), C.byref(h), C.byref(nb)), "smem_gpu_memory")
        return {"index_bytes": ix.value, "batch_device_bytes": d.value, "batch_pinned_bytes": h.value,
                "batches": nb.value}

    def fault(self) -> tuple:
        """(0 | 1 runtime fault | 2 injected sticky fault, message) -- smem_gpu_fault"""
        buf = C.create_string_buffer(512)
        f = load().smem_gpu_fault(self._h, buf, 512)
        return f, buf.value.decode(errors="replace")

    def reserve_slots(self, n_slots: int, reads_per_slot: int, max_len: int) -> None:
        """Pre-size collect_ex worker slots in the background (smem_gpu_reserve_slots)."""
        _check(load().smem_gpu_reserve_slots(self._h, n_slots, reads_per_slot, max_len), "smem_gpu_reserve_slots")

    def batch(self, max_reads: int, max_bases: int, max_len: int) -> "Batch":
        return Batch(self, max_reads, max_bases, max_len)

    def seed_stream(self, codes: np.ndarray, offs: np.ndarray, opt: "Options" = None, chunk_reads: int = 1 << 20,
                    workers: int = 3, pairs: bool = False, collect: bool = False, packed: bool = False,
                    release: bool = False) -> tuple:
        """Stream a read set through smem_gpu_seed_stream (chunks of
        chunk_reads, `workers` host workers each with its own batch and HIP
        stream; packed: 16-B wire entries; release: free the workers'
        batches instead of keeping them for the next call).  Returns (stats
        dict, per-chunk Results in chunk order when collect else None)."""
        lib = load()
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        o = (opt or Options()).c()
        st = StreamStats()
        got = {}
        err = []

        def on_chunk(ctx, chunk, first, n, bh):
            try:
                got[int(chunk)] = _results_of(lib, bh, n, packed)
                return 0
            except Exception as e:  # surfaced after the stream returns
                err.append(e)
                return -5

        cb = CHUNK_FN(on_chunk) if collect else None
        rc = lib.smem_gpu_seed_stream(self._h, offs.size - 1, codes.ctypes.data, offs.ctypes.data, C.byref(o),
                                      int(chunk_reads), int(workers), (1 if pairs else 0) | (2 if packed else 0) | (4 if release else 0),
                                      C.cast(cb, C.c_void_p) if cb else None, None, C.byref(st))
        if err:
            raise err[0]
        _check(rc, "smem_gpu_seed_stream")
        stats = {k: getattr(st, k) for k, _ in StreamStats._fields_}
        return stats, ([got[k] for k in sorted(got)] if collect else None)

    def ksw_extend(self, kb) -> tuple:
        """ksw_extend2 (software/ksw.c:379) of every task of a synth.KswBatch on
        this device: (results as synth.KSW_RESULT, kernel ms)."""
        from . import synth
        lib = load()
        tasks = np.ascontiguousarray(kb.tasks, dtype=synth.KSW_TASK)
        q = np.ascontiguousarray(kb.q, dtype=np.uint8)
        t = np.ascontiguousarray(kb.t, dtype=np.uint8)
        o = KswOptT()
        for i, v in enumerate(np.asarray(kb.mat, dtype=np.int8)):
            o.mat[i] = int(v)
        o.o_del, o.e_del, o.o_ins, o.e_ins = kb.o_del, kb.e_del, kb.o_ins, kb.e_ins
        out = np.zeros(max(tasks.size, 1), dtype=synth.KSW_RESULT)
        ms = C.c_double()
        _check(lib.smem_ksw_extend(self._h, tasks.size, tasks.ctypes.data, q.ctypes.data, q.size, t.ctypes.data,
                                   t.size, C.byref(o), out.ctypes.data, C.byref(ms)), "smem_ksw_extend")
        return out[:tasks.size], ms.value

    def ksw_align2(self, kb) -> tuple:
        """ksw_align2 (software/ksw.c:342) of every KSWA_TASK of a synth.KswBatch
        on this device: (results as synth.KSWA_RESULT, kernel ms)."""
        from . import synth
        lib = load()
        tasks = np.ascontiguousarray(kb.tasks, dtype=synth.KSWA_TASK)
        q = np.ascontiguousarray(kb.q, dtype=np.uint8)
        t = np.ascontiguousarray(kb.t, dtype=np.uint8)
        o = KswOptT()
        for i, v in enumerate(np.asarray(kb.mat, dtype=np.int8)):
            o.mat[i] = int(v)
        o.o_del, o.e_del, o.o_ins, o.e_ins = kb.o_del, kb.e_del, kb.o_ins, kb.e_ins
        out = np.zeros(max(tasks.size, 1), dtype=synth.KSWA_RESULT)
        ms = C.c_double()
        _check(lib.smem_ksw_align2(self._h, tasks.size, tasks.ctypes.data, q.ctypes.data, q.size, t.ctypes.data,
                                   t.size, C.byref(o), out.ctypes.data, C.byref(ms)), "smem_ksw_align2")
        return out[:tasks.size], ms.value

    def load_pac(self, pac, l_pac: int) -> None:
        """Keep the 2-bit .pac resident in HBM (smem_gpu_load_pac)."""
        pac = np.ascontiguousarray(pac, dtype=np.uint8)
        if pac.size < (l_pac + 3) // 4:
            raise SmemError("load_pac: pac holds fewer than (l_pac + 3) / 4 bytes")
        _check(load().smem_gpu_load_pac(self._h, pac.ctypes.data, int(l_pac)), "smem_gpu_load_pac")

    def chain2aln(self, pac, l_pac: int, codes, offs, chains, chain_off, seeds, opt) -> tuple:
        """mem_chain2aln_short / mem_chain2aln of every chain of every read
        (software/bwamem.c:1452-1460) on this device.  opt is a ctypes struct
        laid out as smem_aln_opt_t.  Returns (regions as 64-byte smem_alnreg_t
        records, reg_off[n_reads + 1], kernel ms)."""
        lib = load()
        if pac is not None:
            pac = np.ascontiguousarray(pac, dtype=np.uint8)
            if pac.size < (int(l_pac) + 3) // 4:
                raise SmemError("chain2aln: pac holds fewer than (l_pac + 3) / 4 bytes")
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        chain_off = np.ascontiguousarray(chain_off, dtype=np.uint64)
        chains = np.ascontiguousarray(chains, dtype=CHAIN_DT)
        seeds = np.ascontiguousarray(seeds, dtype=SEED_DT)
        if chain_off.size != offs.size or (chain_off.size and int(chain_off[-1]) > chains.size):
            raise SmemError("chain2aln: chain_off must have n_reads + 1 entries within chains")
        n = offs.size - 1
        cap = int(chains["n"].sum()) if chains.size else 0
        regs = np.zeros(max(cap, 1) * 64, dtype=np.uint8)
        reg_off = np.zeros(n + 1, dtype=np.uint64)
        ms = C.c_double()
        _check(lib.smem_chain2aln(self._h, n, codes.ctypes.data, offs.ctypes.data, chains.ctypes.data,
                                  chain_off.ctypes.data, seeds.ctypes.data, seeds.size,
                                  pac.ctypes.data if pac is not None else None, l_pac,
                                  C.byref(opt), regs.ctypes.data, reg_off.ctypes.data, C.byref(ms)), "smem_chain2aln")
        return regs[:int(reg_off[-1]) * 64], reg_off, ms.value

    def close(self) -> None:
        if self._h:
            load().smem_gpu_shutdown(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Batch:
    """A worker's device-resident reads and results (smem_batch_*)."""

    def __init__(self, gpu: Gpu, max_reads: int, max_bases: int, max_len: int):
        self._gpu = gpu
        self._h = C.c_void_p()
        _check(load().smem_batch_create(gpu._h, max_reads, max_bases, max_len, C.byref(self._h)), "smem_batch_create")

    def set_reads(self, codes: np.ndarray, offs: np.ndarray) -> None:
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        self._keep = (codes, offs)
        _check(load().smem_batch_set_reads_packed(self._h, offs.size - 1, codes.ctypes.data, offs.ctypes.data),
               "smem_batch_set_reads_packed")

    @property
    def n_reads(self) -> int:
        return int(self._keep[1].size - 1)

    def run(self, opt: Options = Options()) -> None:
        o = opt.c()
        _check(load().smem_batch_run(self._h, C.byref(o)), "smem_batch_run")

    def memory(self) -> tuple:
        """(device bytes, pinned host bytes) this batch holds (smem_batch_memory)."""
        d, h = C.c_uint64(), C.c_uint64()
        _check(load().smem_batch_memory(self._h, C.byref(d), C.byref(h)), "smem_batch_memory")
        return d.value, h.value

    def stats(self) -> dict:
        s = BatchStats()
        _check(load().smem_batch_stats(self._h, C.byref(s)), "smem_batch_stats")
        return {k: getattr(s, k) for k, _ in BatchStats._fields_}

    def sa(self, min_seed_len: int = 19, max_occ: int = 10000) -> None:
        """bwt_sa of every seed occurrence of the last run (smem_batch_sa)."""
        _check(load().smem_batch_sa(self._h, min_seed_len, max_occ), "smem_batch_sa")

    def chain(self, l_pac: int, w: int = 100, max_chain_gap: int = 10000, mask_level: float = 0.5,
              drop_ratio: float = 0.5, filter: bool = True) -> None:
        """mem_chain (+ mem_chain_flt) of every read of the last run, over
        the positions of the last sa() (smem_batch_chain)."""
        o = ChainOptT(w, max_chain_gap, mask_level, drop_ratio, int(bool(filter)))
        _check(load().smem_batch_chain(self._h, int(l_pac), C.byref(o)), "smem_batch_chain")

    def chain2aln(self, opt) -> None:
        """mem_chain2aln_short / mem_chain2aln of every chain of the last
        chain(filter=True), over the chains in HBM and the resident .pac
        (smem_batch_chain2aln); opt is laid out as smem_aln_opt_t."""
        _check(load().smem_batch_chain2aln(self._h, C.byref(opt)), "smem_batch_chain2aln")

    def debug_words(self, n_words: int) -> np.ndarray:
        out = np.zeros(n_words, dtype=np.uint64)
        rc = load().smem_batch_debug(self._h, out.ctypes.data, n_words)
        if rc < 0:
            _check(rc, "smem_batch_debug")
        return out[:rc]

    def fetch(self, mask: int | None = None) -> Results:
        """Copy the outputs back (smem_batch_fetch: every stage that ran; with
        `mask`, smem_batch_fetch_mask: only the FETCH_* outputs named) and
        return copies of them."""
        lib = load()
        if mask is None:
            _check(lib.smem_batch_fetch(self._h), "smem_batch_fetch")
        else:
            _check(lib.smem_batch_fetch_mask(self._h, int(mask)), "smem_batch_fetch_mask")
        n = int(self._keep[1].size - 1)
        if mask is None or mask & FETCH_INTV:
            res = _results_of(lib, self._h, n)
        else:
            res = Results(None, None, None, None)
        ni = int(res.intv_off[-1]) if res.intv_off is not None else int(self.stats()["n_intv"])
        pos = C.POINTER(C.c_uint64)()
        oo = C.POINTER(C.c_uint64)()
        no = C.c_uint64()
        if lib.smem_batch_sa_results(self._h, C.byref(pos), C.byref(oo), C.byref(no)) == 0:
            n_occ = int(no.value)
            res.occ_off = np.ctypeslib.as_array(oo, shape=(ni + 1,)).copy()
            res.sa_pos = np.ctypeslib.as_array(pos, shape=(max(n_occ, 1),))[:n_occ].copy()
        ch, sd = C.c_void_p(), C.c_void_p()
        cho = C.POINTER(C.c_uint64)()
        nch, nsd = C.c_uint64(), C.c_uint64()
        if lib.smem_batch_chain_results(self._h, C.byref(ch), C.byref(cho), C.byref(sd), C.byref(nch),
                                        C.byref(nsd)) == 0:
            nc, ns = int(nch.value), int(nsd.value)
            res.chain_off = np.ctypeslib.as_array(cho, shape=(n + 1,)).copy()
            res.chains = np.frombuffer((C.c_char * (max(nc, 1) * CHAIN_DT.itemsize)).from_address(ch.value),
                                       dtype=CHAIN_DT)[:nc].copy()
            res.seeds = np.frombuffer((C.c_char * (max(ns, 1) * SEED_DT.itemsize)).from_address(sd.value),
                                      dtype=SEED_DT)[:ns].copy()
        rg = C.c_void_p()
        ro = C.POINTER(C.c_uint64)()
        nr = C.c_uint64()
        if lib.smem_batch_aln_results(self._h, C.byref(rg), C.byref(ro), C.byref(nr)) == 0:
            k = int(nr.value)
            res.reg_off = np.ctypeslib.as_array(ro, shape=(n + 1,)).copy()
            res.regs = np.frombuffer((C.c_char * (max(k, 1) * 64)).from_address(rg.value), dtype=np.uint8)[:k * 64].copy()
        return res

    def close(self) -> None:
        if self._h:
            load().smem_batch_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def unpack_pintv(p: np.ndarray) -> np.ndarray:
    """(N, 4) uint32 smem_pintv_t entries -> (N, 4) uint64 bwtintv_t (smem_pintv_unpack)."""
    p = p.astype(np.uint64)
    w = p[:, 3]
    out = np.empty((p.shape[0], 4), dtype=np.uint64)
    out[:, 0] = (w & np.uint64(3)) << np.uint64(32) | p[:, 0]
    out[:, 1] = ((w >> np.uint64(2)) & np.uint64(3)) << np.uint64(32) | p[:, 1]
    out[:, 2] = ((w >> np.uint64(4)) & np.uint64(3)) << np.uint64(32) | p[:, 2]
    out[:, 3] = ((w >> np.uint64(6)) & np.uint64(8191)) << np.uint64(32) | (w >> np.uint64(19))
    return out


def _results_of(lib, bh, n: int, packed: bool = False) -> Results:
    """Copies of a fetched batch's interval lists (smem_batch_results, or the
    packed view unpacked)."""
    iv = C.POINTER(Intv)()
    pv = C.c_void_p()
    io = C.POINTER(C.c_uint64)()
    cn = C.POINTER(C.c_uint32)()
    co = C.POINTER(C.c_uint64)()
    if packed:
        _check(lib.smem_batch_results_packed(bh, C.byref(pv), C.byref(io), C.byref(cn), C.byref(co)),
               "smem_batch_results_packed")
    else:
        _check(lib.smem_batch_results(bh, C.byref(iv), C.byref(io), C.byref(cn), C.byref(co)), "smem_batch_results")
    intv_off = np.ctypeslib.as_array(io, shape=(n + 1,)).copy()
    call_off = np.ctypeslib.as_array(co, shape=(n + 1,)).copy()
    ni, nc = int(intv_off[-1]), int(call_off[-1])
    if packed:
        raw = np.ctypeslib.as_array(C.cast(pv, C.POINTER(C.c_uint32)), shape=(max(ni, 1) * 4,))[:ni * 4]
        intv = unpack_pintv(raw.reshape(ni, 4))
    else:
        intv = (np.ctypeslib.as_array(C.cast(iv, C.POINTER(C.c_uint64)), shape=(max(ni, 1) * 4,))[:ni * 4]
                .reshape(ni, 4).copy())
    call_n = np.ctypeslib.as_array(cn, shape=(max(nc, 1),))[:nc].copy()
    return Results(intv, intv_off, call_n, call_off)


def seed(gpu: Gpu, codes: np.ndarray, offs: np.ndarray, opt: Options = Options()) -> Results:
    """Seed all reads on the GPU (one batch) and return the results."""
    offs = np.asarray(offs, dtype=np.uint64)
    lens = np.diff(offs)
    b = gpu.batch(max(1, offs.size - 1), max(1, int(offs[-1] - offs[0])), max(1, int(lens.max()) if lens.size else 1))
    try:
        b.set_reads(codes, offs)
        b.run(opt)
        return b.fetch()
    finally:
        b.close()

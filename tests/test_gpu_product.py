"""The entry points the reference binding (integration/patches) drives per
kt_for_batch worker batch: smem_gpu_init_devices (the index, .sa and .pac on
several device contexts, uploaded side by side), smem_gpu_collect_ex (a
batch per worker slot, results left in HBM) and smem_batch_fetch_mask (only
the outputs the caller reads cross PCIe).

Bar: the same bits as the oracle / the full fetch.  CPU tests cover the
device-list parser (no device needed for an explicit list)."""
import ctypes as C
import threading

import numpy as np
import pytest

from oracle import oracle


def _lib():
    import smemgpu
    return smemgpu.load()


def _parse(spec):
    lib = _lib()
    out = (C.c_int * 16)()
    n = lib.smem_gpu_parse_devices(None if spec is None else spec.encode(), out, 16)
    return n, list(out[:max(n, 0)])


def test_parse_devices_explicit(built):
    assert _parse("0") == (1, [0])
    assert _parse("0,0") == (2, [0, 0])
    assert _parse("3,1,7") == (3, [3, 1, 7])
    for bad in ("x", "1,,2", "1,", "-1", "1;2"):
        n, _ = _parse(bad)
        assert n < 0, bad
    lib = _lib()
    out = (C.c_int * 2)()
    assert lib.smem_gpu_parse_devices(b"0,1,2", out, 2) < 0   # more than max_devices


def test_parse_devices_default_without_gpu(built):
    """The empty spec means every visible device: none here is an error."""
    import smemgpu
    if smemgpu.device_count() > 0:
        pytest.skip("a GPU is visible")
    n, _ = _parse(None)
    assert n == -4  # SMEM_E_DEVICE


@pytest.fixture(scope="module")
def world(gpu_device):
    import smemgpu
    from smemgpu import synth
    g = synth.make_genome(400_000, seed=61, repeat_frac=0.4, n_families=4, exact_frac=0.01, tandem_frac=0.01)
    idx, sa = smemgpu.Index.build_sa(g.codes, sa_intv=32)
    reads = synth.concat_reads([synth.make_reads(g.codes, 3000, 150, seed=62, sub_rate=0.02, n_rate=0.002),
                                synth.make_reads(g.codes, 600, (19, 300), seed=63, sub_rate=0.03, random_frac=0.1)])
    oi = oracle.OracleIndex(words=idx.words, primary=idx.primary, L2=idx.L2)
    want, _, _ = oracle.seed(oi, reads.codes, reads.offs)
    oi.close()
    return dict(g=g, idx=idx, sa=sa, reads=reads, want=want)


def _same_reads(got, want):
    """[read][call] -> (n, 4) arrays, equal bit for bit."""
    assert len(got) == len(want)
    for i, (a, b) in enumerate(zip(got, want)):
        assert len(a) == len(b), i
        for x, y in zip(a, b):
            assert np.array_equal(x, y), i


def _read_lists(reads, i):
    a, b = int(reads.offs[i]), int(reads.offs[i + 1])
    return np.ascontiguousarray(reads.codes[a:b])


def _collect(lib, g, slot, reads, lo, hi, flags=0):
    """smem_gpu_collect_ex of reads [lo, hi) -> (batch handle, the read arrays kept alive)."""
    n = hi - lo
    arrs = [_read_lists(reads, i) for i in range(lo, hi)]
    seq = (C.c_void_p * max(n, 1))(*[a.ctypes.data for a in arrs])
    lens = (C.c_int * max(n, 1))(*[a.size for a in arrs])
    import smemgpu
    o = smemgpu.Options().c()
    bh = C.c_void_p()
    rc = lib.smem_gpu_collect_ex(g, slot, n, seq, lens, C.byref(o), flags, C.byref(bh))
    return rc, bh, arrs


@pytest.mark.gpu
def test_collect_ex_slots_across_threads(world):
    """Worker slots as bwa mem uses them: every chunk starts new threads, and
    thread t of a chunk takes slot t; each slot's batch is reused (and grown)
    by whichever thread holds it.  Every batch's lists == the oracle's."""
    import smemgpu
    from smemgpu.lib import _results_of
    from smemgpu import synth
    lib = _lib()
    gpu = smemgpu.Gpu(world["idx"], device=0)
    reads, want = world["reads"], world["want"]
    got = {}
    errs = []
    # three "chunks", each cut into batches of different sizes dealt to 4 worker threads
    for chunk, bsz in enumerate((97, 400, 1500)):
        bounds = [(a, min(a + bsz, reads.n)) for a in range(0, reads.n, bsz)]

        def worker(t):
            try:
                for k in range(t, len(bounds), 4):
                    lo, hi = bounds[k]
                    rc, bh, keep = _collect(lib, gpu._h, t, reads, lo, hi)
                    assert rc == 0, smemgpu.lib.ERRORS.get(rc, rc)
                    res = _results_of(lib, bh, hi - lo)
                    got[(chunk, lo)] = res.to_smgo()
            except Exception as e:  # surfaced below
                errs.append(e)

        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs[0]
        # reassemble the chunk's per-batch SMGO streams and compare with the oracle's
        recs = []
        for lo, hi in bounds:
            recs.extend(synth.read_smgo(got[(chunk, lo)]))
        _same_reads(recs, synth.read_smgo(want))
    gpu.close()


@pytest.mark.gpu
def test_collect_ex_no_fetch_then_stages(world):
    """SMEM_COLLECT_NO_FETCH leaves the lists in HBM; sa -> chain(filter) ->
    chain2aln run on them; fetch_mask(REGS) copies only the regions, which
    equal the full fetch's; views of outputs not fetched, and masks naming a
    stage that has not run, are refused."""
    import smemgpu
    lib = _lib()
    g, reads = world["g"], world["reads"]
    gpu = smemgpu.Gpu(world["idx"], device=0)
    try:
        gpu.load_sa(world["sa"])
        pac = _pack(g.codes)
        gpu.load_pac(pac, g.codes.size)
        rc, bh, keep = _collect(lib, gpu._h, 0, reads, 0, reads.n, flags=smemgpu.lib.COLLECT_NO_FETCH)
        assert rc == 0
        iv = C.POINTER(smemgpu.lib.Intv)()
        off = C.POINTER(C.c_uint64)()
        assert lib.smem_batch_results(bh, C.byref(iv), C.byref(off), None, None) != 0   # nothing fetched
        assert lib.smem_batch_fetch_mask(bh, smemgpu.lib.FETCH_REGS) != 0                # no regions yet
        assert lib.smem_batch_fetch_mask(bh, 16) != 0                                    # unknown bit
        assert lib.smem_batch_sa(bh, 19, 500) == 0
        co = smemgpu.lib.ChainOptT(100, 10000, 0.5, 0.5, 1)
        assert lib.smem_batch_chain(bh, int(g.codes.size), C.byref(co)) == 0
        opt = oracle.aln_opt()
        assert lib.smem_batch_chain2aln(bh, C.byref(opt)) == 0
        assert lib.smem_batch_fetch_mask(bh, smemgpu.lib.FETCH_REGS) == 0
        rg = C.c_void_p()
        ro = C.POINTER(C.c_uint64)()
        nr = C.c_uint64()
        assert lib.smem_batch_aln_results(bh, C.byref(rg), C.byref(ro), C.byref(nr)) == 0
        n_regs = int(nr.value)
        regs_only = np.frombuffer((C.c_char * (max(n_regs, 1) * 64)).from_address(rg.value), dtype=np.uint8)[
            :n_regs * 64].copy()
        roff = np.ctypeslib.as_array(ro, shape=(reads.n + 1,)).copy()
        assert lib.smem_batch_results(bh, C.byref(iv), C.byref(off), None, None) != 0   # intervals not copied
        assert lib.smem_batch_chain_results(bh, None, None, None, None, None) != 0      # chains not copied
        assert lib.smem_batch_fetch(bh) == 0                                             # now everything
        from smemgpu.lib import _results_of
        res = _results_of(lib, bh, reads.n)
        assert res.to_smgo() == world["want"]
        assert lib.smem_batch_aln_results(bh, C.byref(rg), C.byref(ro), C.byref(nr)) == 0
        full = np.frombuffer((C.c_char * (max(n_regs, 1) * 64)).from_address(rg.value), dtype=np.uint8)[
            :n_regs * 64].copy()
        assert int(nr.value) == n_regs and n_regs > reads.n
        assert np.array_equal(full, regs_only)
        assert np.array_equal(np.ctypeslib.as_array(ro, shape=(reads.n + 1,)), roff)
    finally:
        gpu.close()


def _pack(codes):
    c = np.asarray(codes, dtype=np.uint8)
    out = np.zeros((c.size + 3) // 4, dtype=np.uint8)
    for k in range(4):
        part = c[k::4]
        out[:part.size] |= (np.minimum(part, 3) << (6 - 2 * k)).astype(np.uint8)
    return out


@pytest.mark.gpu
def test_init_devices_two_contexts(world):
    """smem_gpu_init_devices on "0,0": two contexts, each with the index, .sa
    and .pac resident; both seed the same lists; a bad device shuts down what
    was opened and zeroes the handles."""
    import smemgpu
    from smemgpu.lib import _results_of
    lib = _lib()
    idx, sa, g, reads = world["idx"], world["sa"], world["g"], world["reads"]
    pac = _pack(g.codes)
    words = idx.words
    L2 = (C.c_uint64 * 5)(*[int(v) for v in idx.L2])
    hs = (C.c_void_p * 2)()
    devs = (C.c_int * 2)(0, 0)
    rc = lib.smem_gpu_init_devices(hs, 2, devs, words.ctypes.data, words.size, idx.primary, L2, C.byref(sa._raw),
                                   pac.ctypes.data, int(g.codes.size))
    assert rc == 0, lib.smem_strerror(rc)
    try:
        assert hs[0] and hs[1] and hs[0] != hs[1]
        for h in (hs[0], hs[1]):
            rc, bh, keep = _collect(lib, h, 0, reads, 0, 800)
            assert rc == 0
            assert lib.smem_batch_sa(bh, 19, 500) == 0   # the .sa is resident on this context
            res = _results_of(lib, bh, 800)
            from smemgpu import synth
            _same_reads(synth.read_smgo(res.to_smgo()), synth.read_smgo(world["want"])[:800])
    finally:
        lib.smem_gpu_shutdown(hs[0])
        lib.smem_gpu_shutdown(hs[1])
    bad = (C.c_int * 2)(0, 4095)
    rc = lib.smem_gpu_init_devices(hs, 2, bad, words.ctypes.data, words.size, idx.primary, L2, None, None, 0)
    assert rc != 0 and not hs[0] and not hs[1]
    assert b"device 4095" in lib.smem_strerror(rc)


def _slot_run(lib, gpu, t, reads, lo, hi):
    """One worker batch through every stage on slot t, as mem_batch_gpu runs it:
    (seeding lists as SMGO, the regions' bytes, their per-read offsets)."""
    import smemgpu
    from smemgpu.lib import _results_of
    rc, bh, keep = _collect(lib, gpu._h, t, reads, lo, hi, flags=smemgpu.lib.COLLECT_NO_FETCH)
    assert rc == 0, smemgpu.lib.ERRORS.get(rc, rc)
    assert lib.smem_batch_sa(bh, 19, 500) == 0
    co = smemgpu.lib.ChainOptT(100, 10000, 0.5, 0.5, 1)
    assert lib.smem_batch_chain(bh, int(gpu._l_pac), C.byref(co)) == 0
    opt = smemgpu.aln_opt()
    assert lib.smem_batch_chain2aln(bh, C.byref(opt)) == 0
    assert lib.smem_batch_fetch(bh) == 0
    smgo = _results_of(lib, bh, hi - lo).to_smgo()
    rg, ro, nr = C.c_void_p(), C.POINTER(C.c_uint64)(), C.c_uint64()
    assert lib.smem_batch_aln_results(bh, C.byref(rg), C.byref(ro), C.byref(nr)) == 0
    n = int(nr.value)
    regs = np.frombuffer((C.c_char * (max(n, 1) * 64)).from_address(rg.value), dtype=np.uint8)[:n * 64].copy()
    return smgo, regs, np.ctypeslib.as_array(ro, shape=(hi - lo + 1,)).copy()


@pytest.mark.gpu
@pytest.mark.parametrize("arena", ["1", "0"])
def test_reserved_slots_every_stage(world, monkeypatch, arena):
    """smem_gpu_reserve_slots (what the patched main_mem calls for -t / -b):
    every slot's buffers carved from one device and one pinned block
    (SMEM_GPU_ARENA=1, the default) or allocated one by one (0), slot 0's
    warm-up over reads cut from the resident .pac.  Four threads then run
    worker batches on their slots through every stage, some larger than the
    reservation (such a slot's batch is re-created at its size): seeding lists
    equal the oracle's, regions equal those of an unreserved handle's batches."""
    import smemgpu
    from smemgpu import synth
    monkeypatch.setenv("SMEM_GPU_ARENA", arena)
    lib = _lib()
    g, reads = world["g"], world["reads"]
    pac = _pack(g.codes)

    def open_gpu():
        gpu = smemgpu.Gpu(world["idx"], device=0)
        gpu.load_sa(world["sa"])
        gpu.load_pac(pac, g.codes.size)
        gpu._l_pac = g.codes.size
        return gpu

    bounds, a, k = [], 0, 0
    while a < reads.n:  # 350- and 450-read batches: the larger outgrow the 400-read slots
        b = min(a + (350, 450)[k % 2], reads.n)
        bounds.append((a, b))
        a, k = b, k + 1
    ref = open_gpu()  # no reservation: every slot created on first use
    try:
        want = {lo: _slot_run(lib, ref, 0, reads, lo, hi) for lo, hi in bounds}
    finally:
        ref.close()
    gpu = open_gpu()
    try:
        gpu.reserve_slots(4, 400, 300)
        got, errs = {}, []

        def worker(t):
            try:
                for k in range(t, len(bounds), 4):
                    lo, hi = bounds[k]
                    got[lo] = _slot_run(lib, gpu, t, reads, lo, hi)
            except Exception as e:  # surfaced below
                errs.append(e)

        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs[0]
        recs = []
        for lo, hi in bounds:
            recs.extend(synth.read_smgo(got[lo][0]))
            assert np.array_equal(got[lo][1], want[lo][1]) and np.array_equal(got[lo][2], want[lo][2]), lo
        _same_reads(recs, synth.read_smgo(world["want"]))
        m = gpu.memory()
        assert m["batches"] == 4 and m["batch_device_bytes"] > 0 and m["batch_pinned_bytes"] > 0, m
    finally:
        gpu.close()

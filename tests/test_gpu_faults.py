"""The library's failure contract and the binding's reject -> CPU path
(include/smem_gpu.h, "Failure contract"; the reference's semantics:
software/bwt.c:686-717, a refused batch computed on the CPU).

SMEM_GPU_FAIL=<stage>:<k>[:sticky|:hip=<code>] makes every k-th call of a stage return
SMEM_E_DEVICE after its work is enqueued and before it is waited for, so the
drain on the way out of the call is what keeps that work from landing after
the caller resumed.  ":sticky" also marks the device faulted, as a real HIP
runtime failure does: every later call is refused without touching the GPU.

* library level: the refused call returns SMEM_E_DEVICE, the next call on the
  same batch (non-sticky) is bit-exact against the oracle; after a sticky
  fault every entry point returns SMEM_E_DEVICE ("faulted earlier");
* bwa level: the reference's `bwa mem` with the integration patch, failures
  injected at every stage: the refused batches take the CPU path and the SAM
  is byte-identical to the reference's golden SAM (SE and PE).
"""
import os

import numpy as np
import pytest

from oracle import oracle
from test_bwa_integration import _golden, _need_bwa, _run, _same, indexed  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu


@pytest.fixture
def fail_env():
    """Set SMEM_GPU_FAIL for this process (the library reads it per call)."""
    old = os.environ.get("SMEM_GPU_FAIL")

    def setter(v):
        if v is None:
            os.environ.pop("SMEM_GPU_FAIL", None)
        else:
            os.environ["SMEM_GPU_FAIL"] = v
    yield setter
    setter(old)


@pytest.fixture(scope="module")
def small(gpu_device):
    import smemgpu
    from smemgpu import synth
    genome = synth.make_genome(200_000, seed=41)
    idx, sa = smemgpu.Index.build_sa(genome.codes)
    ref = oracle.OracleIndex(words=idx.words, primary=idx.primary, L2=idx.L2)
    reads = synth.make_reads(genome.codes, 600, 150, seed=42)
    want, _, _ = oracle.seed(ref, reads.codes, reads.offs, threads=4)
    return dict(genome=genome, idx=idx, sa=sa, reads=reads, want=want)


@pytest.mark.parametrize("stage", ["upload", "seed", "fetch"])
def test_injected_failure_then_clean_rerun(small, gpu_device, fail_env, stage):
    """A refused call returns SMEM_E_DEVICE; the device is not faulted (not
    sticky), and the same batch then reruns bit-exact."""
    import smemgpu
    gpu = smemgpu.Gpu(small["idx"], device=gpu_device)
    try:
        r = small["reads"]
        b = gpu.batch(r.n, int(r.codes.size), int(r.lens.max()))
        fail_env(f"{stage}:1")  # every call of the stage fails
        with pytest.raises(smemgpu.SmemError, match="SMEM_E_DEVICE.*injected"):
            b.set_reads(r.codes, r.offs)
            b.run()
            b.fetch()
        fail_env(None)
        b.set_reads(r.codes, r.offs)
        b.run()
        assert b.fetch().to_smgo() == small["want"]
        assert gpu.fault()[0] == 0
        b.close()
    finally:
        fail_env(None)
        gpu.close()


def test_sticky_fault_refuses_every_later_call(small, gpu_device, fail_env):
    """A runtime failure marks the device faulted: every later entry point is
    refused at once (the caller's CPU path takes over), batch creation too."""
    import smemgpu
    gpu = smemgpu.Gpu(small["idx"], device=gpu_device)
    try:
        r = small["reads"]
        b = gpu.batch(r.n, int(r.codes.size), int(r.lens.max()))
        b.set_reads(r.codes, r.offs)
        fail_env("seed:1:sticky")
        with pytest.raises(smemgpu.SmemError, match="SMEM_E_DEVICE"):
            b.run()
        fail_env(None)
        f, msg = gpu.fault()
        assert f == 2 and "injected" in msg, (f, msg)  # 2: injected (1 would be a real runtime fault)
        for call in (lambda: b.set_reads(r.codes, r.offs), lambda: b.run(),
                     lambda: gpu.batch(10, 1000, 100)):
            with pytest.raises(smemgpu.SmemError, match="faulted earlier"):
                call()
        b.close()
    finally:
        fail_env(None)
        gpu.close()


@pytest.mark.parametrize("code,sticky", [(9, False), (1, False), (719, True), (700, True)])
def test_injected_hip_error_classification(small, gpu_device, fail_env, code, sticky):
    """A HIP runtime error goes through the library's classification: a
    launch-configuration or argument error (hipErrorInvalidConfiguration 9,
    hipErrorInvalidValue 1) refuses that one call and leaves the device usable
    (the same batch reruns bit-exact); a kernel fault (hipErrorLaunchFailure
    719, hipErrorIllegalAddress 700) marks the device faulted for good."""
    import smemgpu
    gpu = smemgpu.Gpu(small["idx"], device=gpu_device)
    try:
        r = small["reads"]
        b = gpu.batch(r.n, int(r.codes.size), int(r.lens.max()))
        b.set_reads(r.codes, r.offs)
        fail_env(f"seed:1:hip={code}")
        with pytest.raises(smemgpu.SmemError, match="SMEM_E_DEVICE"):
            b.run()
        fail_env(None)
        f, msg = gpu.fault()
        if sticky:
            assert f == 1 and "injected" in msg, (f, msg)
            with pytest.raises(smemgpu.SmemError, match="faulted earlier"):
                b.run()
        else:
            assert f == 0, (f, msg)
            b.set_reads(r.codes, r.offs)
            b.run()
            assert b.fetch().to_smgo() == small["want"]
        b.close()
    finally:
        fail_env(None)
        gpu.close()


def test_admission_bound_concurrent_workers(small, gpu_device):
    """More host workers than admitted calls (max_active 2, 6 threads): every
    worker's results are bit-exact; the waiting workers are admitted in turn.
    A warm-up at max_active 4 makes four stream pairs first; lowering the
    limit to 2 then holds (leases are counted against it, not pairs)."""
    import threading
    import smemgpu
    gpu = smemgpu.Gpu(small["idx"], device=gpu_device)
    r = small["reads"]
    errs, ok = [], []

    def worker(reps):
        try:
            b = gpu.batch(r.n, int(r.codes.size), int(r.lens.max()))
            for _ in range(reps):
                b.set_reads(r.codes, r.offs)
                b.run()
                ok.append(b.fetch().to_smgo() == small["want"])
            b.close()
        except Exception as e:  # surfaced below
            errs.append(e)

    assert gpu.max_active() == 8  # the default (SMEM_GPU_MAX_ACTIVE unset)
    for limit, reps in ((4, 1), (2, 3)):
        gpu.set_max_active(limit)
        assert gpu.max_active() == limit
        th = [threading.Thread(target=worker, args=(reps,)) for _ in range(6)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    gpu.close()
    assert not errs, errs[0]
    assert len(ok) == 24 and all(ok)


def test_async_init_devices(small, gpu_device):
    """smem_gpu_init_devices_async: the call returns before the upload; the
    first device call waits for it and the results are bit-exact (two
    contexts on the device, as the binding's "0,0"); a device that does not
    exist is refused before anything runs, as smem_gpu_init_devices does."""
    import smemgpu
    with pytest.raises(smemgpu.SmemError, match="out of range"):
        smemgpu.Gpu.open_async(small["idx"], [gpu_device, 63], sa=small["sa"])
    gs = smemgpu.Gpu.open_async(small["idx"], [gpu_device, gpu_device], sa=small["sa"])
    try:
        r = small["reads"]
        for g in gs:
            assert smemgpu.seed(g, r.codes, r.offs).to_smgo() == small["want"]
            g.wait_ready()
            assert g.fault()[0] == 0
    finally:
        for g in gs:
            g.close()


# every stage, every k-th call; "any:5" spreads over all of them; the sticky
# case faults the device on the first seeding call, so the rest is refused
INJECT = ["upload:2", "seed:2", "sa:3", "chain:2", "aln:2", "fetch:3", "any:5", "seed:2:sticky"]


@pytest.mark.parametrize("kind", ["se", "pe"])
@pytest.mark.parametrize("spec", INJECT)
def test_bwa_injected_failures_sam_identical(indexed, gpu_device, kind, spec):  # noqa: F811
    """bwa-gpu mem with SMEM_GPU_FAIL: the refused worker batches take the CPU
    path (mem_chain ... mem_chain2aln), the others the GPU; the SAM equals the
    reference's golden SAM byte for byte."""
    _need_bwa()
    got, err = _run(indexed["g1"], "g1", kind, 4, 64, env={"SMEM_GPU_FAIL": spec, "SMEM_GPU_TIMES": "1"})
    n_fail = err.count("GPU runtime failure")
    n_batches = err.count("[M::mem_batch_gpu]")
    if "sticky" not in spec:
        assert 0 < n_fail < n_batches, f"{n_fail} of {n_batches} batches refused\n" + err[-2000:]
    else:
        # the faulted context is reported once (not once per refused batch)
        # and every later batch is refused by it, on the CPU path
        assert err.count("GPU context 0 faulted (") == 1, err[-2000:]
        assert "injected failure" in err, err[-2000:]
    _same(got, _golden("g1", kind))

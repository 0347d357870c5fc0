"""Minimal workload for rocprofv3 counter passes: build (or reuse) the index,
seed one batch --launches times.  Meant to run under

    rocprofv3 --pmc <counters> --kernel-include-regex seed_kernel -- python tools/prof_run.py ...
"""
import argparse
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--genome-mbp", type=float, default=3101.804739)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--reads", type=int, default=1_000_000)
    p.add_argument("--read-len", type=int, default=150)
    p.add_argument("--sub", type=float, default=0.02)
    p.add_argument("--lanes-per-cu", type=int, default=0)
    p.add_argument("--launches", type=int, default=1)
    p.add_argument("--variant", type=int, default=0)
    p.add_argument("--cache", default=os.path.join(tempfile.gettempdir(), "smem_bench_cache"))
    a = p.parse_args()
    import smemgpu
    from smemgpu import synth
    os.makedirs(a.cache, exist_ok=True)
    n_bp = int(a.genome_mbp * 1e6)
    key = os.path.join(a.cache, f"genome_{n_bp}_{a.seed}.bwt")
    g = synth.make_genome(n_bp, seed=a.seed, n_chrom=24)
    if not os.path.exists(key):
        smemgpu.Index.build_gpu(g.codes).write(key)
    idx = smemgpu.Index.read(key)
    reads = synth.make_reads(g.codes, a.reads, a.read_len, seed=1000 + a.seed * 7919, sub_rate=a.sub, n_rate=0.001)
    gpu = smemgpu.Gpu(idx, device=0, lanes_per_cu=a.lanes_per_cu, variant=a.variant)
    b = gpu.batch(reads.n, reads.codes.size, int(reads.lens.max()))
    b.set_reads(reads.codes, reads.offs)
    for _ in range(a.launches):
        t = time.time()
        b.run()
        print(f"launch: kernel {b.stats()['kernel_ms']:.3f} ms, wall {1e3 * (time.time() - t):.1f} ms", flush=True)
    b.close()
    gpu.close()


if __name__ == "__main__":
    main()

"""Launch-shape / workload sweep of the seeding kernel on one GPU.

    python tools/sweep.py --genome-mbp 400 --lanes 256,512,1024 --reads 1000000

Builds (or reuses from --cache) the synthetic index, then for each lanes/CU
setting runs the batch a few times and prints kernel ms and reads/s.  Every
configuration is checked against the first one's results (bit-exact).
"""
import argparse
import hashlib
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--genome-mbp", type=float, default=100)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--builder", choices=["gpu", "cpu"], default="gpu")
    p.add_argument("--reads", type=int, default=1_000_000)
    p.add_argument("--read-len", type=int, default=150)
    p.add_argument("--sub", type=float, default=0.02)
    p.add_argument("--lanes", default="256,512,1024")
    p.add_argument("--variants", default="2",
                   help="seeding kernel variants to compare; V:K = variant V with a K-mer table (e.g. 23:12)")
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--cache", default=os.path.join(tempfile.gettempdir(), "smem_bench_cache"))
    a = p.parse_args()
    import smemgpu
    from smemgpu import synth
    os.makedirs(a.cache, exist_ok=True)
    n_bp = int(a.genome_mbp * 1e6)
    key = os.path.join(a.cache, f"genome_{n_bp}_{a.seed}.bwt")
    g = synth.make_genome(n_bp, seed=a.seed, n_chrom=24)
    if not os.path.exists(key):
        t = time.time()
        (smemgpu.Index.build_gpu(g.codes) if a.builder == "gpu" else smemgpu.Index.build(g.codes)).write(key)
        print(f"index built in {time.time() - t:.1f}s", flush=True)
    idx = smemgpu.Index.read(key)
    reads = synth.make_reads(g.codes, a.reads, a.read_len, seed=1000 + a.seed * 7919, sub_rate=a.sub, n_rate=0.001)
    ref_hash = None
    confs = [(v, l) for v in a.variants.split(",") for l in [int(x) for x in a.lanes.split(",")]]
    for vspec, lanes in confs:
        variant, kmer_k = (int(x) for x in (vspec + ":0").split(":")[:2])
        t = time.time()
        gpu = smemgpu.Gpu(idx, device=0, lanes_per_cu=lanes, variant=variant, kmer_k=kmer_k)
        t_init = time.time() - t
        b = gpu.batch(reads.n, reads.codes.size, int(reads.lens.max()))
        b.set_reads(reads.codes, reads.offs)
        b.run()
        h = hashlib.sha256(b.fetch().intv.tobytes()).hexdigest()
        ref_hash = ref_hash or h
        ks = []
        for _ in range(a.reps):
            b.run()
            ks.append(b.stats()["kernel_ms"])
        st = b.stats()
        print(json.dumps({"genome_mbp": a.genome_mbp, "variant": variant, "kmer_k": kmer_k, "init_s": round(t_init, 2),
                          "lanes_per_cu": lanes, "grid": st["grid"],
                          "kernel_ms_min": round(min(ks), 3), "kernel_ms_med": round(float(np.median(ks)), 3),
                          "reads_per_s": round(reads.n / (min(ks) * 1e-3)), "same_result": h == ref_hash}),
              flush=True)
        b.close()
        gpu.close()


if __name__ == "__main__":
    main()

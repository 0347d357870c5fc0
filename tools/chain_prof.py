"""Chaining-stage timing on the bench workload: smem_batch_chain with and
without the filter, and the reads that carry the most seeds / chains.

    python tools/chain_prof.py [--genome-mbp 2000 --reads 1000000]
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--genome-mbp", type=float, default=3101.804739)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--reads", type=int, default=1_000_000)
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--cache", default=os.path.join(tempfile.gettempdir(), "smem_bench_cache"))
    a = p.parse_args()
    import smemgpu
    from smemgpu import synth
    os.makedirs(a.cache, exist_ok=True)
    n_bp = int(a.genome_mbp * 1e6)
    g = synth.make_genome(n_bp, seed=a.seed, n_chrom=24)
    key = os.path.join(a.cache, f"genome_{n_bp}_{a.seed}")
    if not os.path.exists(key + ".bwt"):
        idx, sa = smemgpu.Index.build_sa(g.codes, sa_intv=32, gpu=True)
        idx.write(key + ".bwt")
        sa.write(key + ".sa")
    idx, sa = smemgpu.Index.read(key + ".bwt"), smemgpu.SA.read(key + ".sa")
    reads = synth.make_reads(g.codes, a.reads, 150, seed=1000 + a.seed * 7919, sub_rate=0.02, n_rate=0.001)
    gpu = smemgpu.Gpu(idx)
    gpu.load_sa(sa)
    b = gpu.batch(reads.n, reads.codes.size, 150)
    b.set_reads(reads.codes, reads.offs)
    b.run()
    b.sa(19, 10000)
    out = {}
    for filt in (False, True):
        ms = []
        for _ in range(a.reps):
            b.chain(idx.seq_len // 2, filter=filt)
            ms.append(b.stats()["chain_ms"])
        out[f"filter{int(filt)}_ms"] = ms
    if os.environ.get("SMEM_CHAIN_DBG"):
        d = b.debug_words(256 * 16).reshape(256, 16).astype(np.int64)
        d = d[np.argsort(-(d[:, 9] - d[:, 2]))]
        out["heavy_phases_cycles"] = [dict(total=int(x[9] - x[2]), us=(x[15] - x[14]) / 100.0, read=int(x[0]), seeds=int(x[1]), chains=int(x[4]), insert=int(x[3] - x[2]),
                                           weights=int(x[5] - x[3]), sort=int(x[6] - x[5]), drop=int(x[7] - x[6]),
                                           kept=int(x[8]), tail=int(x[9] - x[7]), replay=int(x[10]), cluster_pass=int(x[11] - x[2]) if x[11] else 0,
                                           n_cand=int(x[12])) for x in d[:16] if x[9]]
    res = b.fetch()
    n_seed = np.array([res.read_sa(i).size for i in range(reads.n)]) if reads.n <= 2_000_000 else None
    n_chain = np.diff(res.chain_off)
    top = np.argsort(-n_seed)[:8]
    out["top_reads"] = [dict(read=int(r), seeds=int(n_seed[r]), chains=int(n_chain[r])) for r in top]
    out["seeds_pctl"] = {q: float(np.percentile(n_seed, q)) for q in (50, 99, 99.9, 99.99)}
    out["reads_over"] = {t: int((n_seed > t).sum()) for t in (64, 256, 1024, 4096)}
    print(json.dumps(out), flush=True)
    b.close()
    gpu.close()


if __name__ == "__main__":
    main()

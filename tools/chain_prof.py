"""Chaining-stage timing on the bench workload: smem_batch_chain with and
without the filter, and the reads that carry the most seeds / chains.

    SMEM_CHAIN_DBG=1 python tools/chain_prof.py [--reps 2] [bench args]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)


def main():
    """the bench's index, reads and options (bench args pass through, e.g.
    --genome-profile human)"""
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--sweep", default="", help="giant_min:lds_rest_kb,... timed with the filter")
    own, rest = p.parse_known_args()
    import torch
    torch.cuda.device_count()  # as bench.py's Dist does, before libsmemgpu touches the device
    import bench
    import smemgpu
    a = bench.parse(rest)
    a.reps = own.reps
    idx, _, sa, codes = bench.get_index(a, 0, lambda: None, 0)
    reads = bench.make_reads(a, 0, codes, 1)
    gpu = smemgpu.Gpu(idx, device=0, lanes_per_cu=a.lanes_per_cu)
    gpu.load_sa(sa)
    b = gpu.batch(reads.n, reads.codes.size, int(reads.lens.max()))
    b.set_reads(reads.codes, reads.offs)
    b.run(smemgpu.Options(min_seed_len=a.min_seed_len))
    b.sa(a.min_seed_len, 10000)
    out = {}
    for filt in (False, True):
        ms = []
        for _ in range(a.reps):
            b.chain(idx.seq_len // 2, filter=filt)
            ms.append(b.stats()["chain_ms"])
        out[f"filter{int(filt)}_ms"] = ms
    for item in [x for x in own.sweep.split(",") if x]:
        gm, lr = item.split(":")
        os.environ["SMEM_CHAIN_GIANT_MIN"] = gm
        os.environ["SMEM_CHAIN_LDS_REST"] = str(int(lr) * 1024)
        ms = []
        for _ in range(a.reps):
            b.chain(idx.seq_len // 2, filter=True)
            ms.append(b.stats()["chain_ms"])
        out[f"sweep_{gm}_{lr}k_ms"] = ms
        print(item, ms, file=sys.stderr, flush=True)
    os.environ.pop("SMEM_CHAIN_GIANT_MIN", None)
    os.environ.pop("SMEM_CHAIN_LDS_REST", None)
    if own.sweep:
        b.chain(idx.seq_len // 2, filter=True)
    if os.environ.get("SMEM_CHAIN_DBG"):
        d = b.debug_words(256 * 32).reshape(256, 32).astype(np.int64)
        d = d[np.argsort(-(d[:, 9] - d[:, 2]))]
        out["heavy_phases_cycles"] = [dict(total=int(x[9] - x[2]), us=(x[15] - x[14]) / 100.0, read=int(x[0]), seeds=int(x[1]), chains=int(x[4]), insert=int(x[3] - x[2]),
                                           weights=int(x[5] - x[3]), sort=int(x[6] - x[5]), drop=int(x[7] - x[6]),
                                           kept=int(x[8]), tail=int(x[9] - x[7]), replay=int(x[10]), cluster_pass=int(x[11] - x[2]) if x[11] else 0,
                                           n_cand=int(x[12]), drop_kept=int(x[13] - x[6]) if x[13] > x[6] else None, in_lds=int(x[23]),
                                           p2_steps=int(x[30]), p2_members=int(x[31]),
                                           combsort=[int(x[16]), int(x[17])], partitions=[int(x[18]), int(x[19])],
                                           sort_parts=int(x[20] - x[5]) if x[20] else None, n_small=int(x[21]),
                                           sort_small=int(x[22] - x[20]) if x[22] else None, sort_close=int(x[24] - x[22]) if x[24] else None,
                                           replay_split=dict(search=int(x[25]), merge=int(x[26]), insert=int(x[27]),
                                                             n_search=int(x[28]), n_insert=int(x[29])) if x[10] else None) for x in d[:16] if x[9]]
        live = d[d[:, 9] > 0]
        out["recorded_phase_sums"] = dict(reads=int(len(live)), total=int((live[:, 9] - live[:, 2]).sum()),
                                          insert=int((live[:, 3] - live[:, 2]).sum()), weights=int((live[:, 5] - live[:, 3]).sum()),
                                          sort=int((live[:, 6] - live[:, 5]).sum()), drop=int((live[:, 7] - live[:, 6]).sum()),
                                          tail=int((live[:, 9] - live[:, 7]).sum()), chains=int(live[:, 4].sum()),
                                          seeds=int(live[:, 1].sum()))
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

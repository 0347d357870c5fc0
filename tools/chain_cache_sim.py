"""How often mem_chain's lower-chain lookups would hit a small direct-mapped
record cache, on the reads with the most seed occurrences.

Sizes the chaining replay's LDS record cache (DESIGN.md §5 chaining): the
replay reads the lower chain's record from HBM on one lane for every seed
(software/bwamem.c:462-499: kb_intervalp, then test_and_merge on that chain);
a write-through cache keyed by chain id would serve repeats from LDS.  The
seeds come from the restatement (oracle/, test infrastructure) on a synthetic
genome; the lower chain is found with a sorted list (exact for distinct chain
positions, an approximation of kbtree's choice among equal ones).

  python tools/chain_cache_sim.py --mbp 100 --reads 300000 --top 30
"""
import argparse
import bisect
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "bwa-mem-harp2_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))

from smemgpu import synth  # noqa: E402
import smemgpu  # noqa: E402
from oracle import oracle  # noqa: E402


def merge(c, rb, qb, ln, w=100, gap=10000, l_pac=None):
    # test_and_merge (software/bwamem.c:334-354): 0 new chain, 1 contained, 2 appended
    pos, last_rb, fq, lq, ll = c
    if qb >= fq and qb + ln <= lq + ll and rb >= pos and rb + ln <= last_rb + ll:
        return 1
    if (last_rb < l_pac or pos < l_pac) and rb >= l_pac:
        return 0
    x, y = qb - lq, rb - last_rb
    if y >= 0 and x - y <= w and y - x <= w and x - ll < gap and y - ll < gap:
        return 2
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mbp", type=float, default=100)
    ap.add_argument("--reads", type=int, default=300000)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--caps", default="64,128,256,512,1024,2048")
    ap.add_argument("--cache", default="/tmp/wp_stats_idx")
    a = ap.parse_args()
    n_bp = int(a.mbp * 1e6)
    g = synth.make_genome(n_bp, seed=1)
    os.makedirs(a.cache, exist_ok=True)
    fb, fs = os.path.join(a.cache, f"uniform_{n_bp}.bwt"), os.path.join(a.cache, f"uniform_{n_bp}.sa")
    if not (os.path.exists(fb) and os.path.exists(fs)):
        idx, sa = smemgpu.Index.build_sa(g.codes, sa_intv=32)
        idx.write(fb)
        sa.write(fs)
    oi, osa = oracle.OracleIndex(fb), oracle.OracleSA(fs)
    r = synth.make_reads(g.codes, a.reads, 150, seed=7)
    data, _, _ = oracle.seed(oi, r.codes, r.offs, threads=8)
    lists = synth.read_smgo(data)
    occ = np.array([sum(int(((x[:, 3] & 0xFFFFFFFF).astype(np.int64) - (x[:, 3] >> 32).astype(np.int64) >= 19).astype(
        np.int64) @ np.where(x[:, 2] <= 10000, x[:, 2], 0).astype(np.int64)) for x in L if x.shape[0]) for L in lists])
    top = np.argsort(-occ)[:a.top]
    caps = [int(c) for c in a.caps.split(",")]
    out = {"mbp": a.mbp, "reads": a.reads, "top_reads": []}
    tot = {c: [0, 0] for c in caps}
    for ri in top:
        counts, k = oracle.sa_queries([lists[ri]], 19, 10000)
        pos = osa.lookup(oi, k)
        seeds, _ = oracle.chain_seeds([lists[ri]], [pos], 19, 10000)
        keys, ids, ch, acc = [], [], [], []
        l_pac = n_bp
        for s in seeds:
            rb, qb, ln = int(s["rbeg"]), int(s["qbeg"]), int(s["len"])
            if rb < l_pac < rb + ln:
                continue
            i = bisect.bisect_right(keys, rb) - 1
            if i >= 0:
                cid = ids[i]
                acc.append(cid)
                m = merge(ch[cid], rb, qb, ln, l_pac=l_pac)
                if m:
                    if m == 2:
                        p, _, fq, _, _ = ch[cid]
                        ch[cid] = (p, rb, fq, qb, ln)
                    continue
            cid = len(ch)
            ch.append((rb, rb, qb, qb, ln))
            acc.append(-1 - cid)  # a creation installs the record
            j = bisect.bisect_right(keys, rb)
            keys.insert(j, rb)
            ids.insert(j, cid)
        rec = {"read": int(ri), "seeds": int(len(seeds)), "chains": len(ch),
               "lookups": sum(1 for x in acc if x >= 0)}
        for c in caps:
            tag = [-1] * c
            hit = look = 0
            for x in acc:
                cid = x if x >= 0 else -1 - x
                if x >= 0:
                    look += 1
                    hit += tag[cid & (c - 1)] == cid
                tag[cid & (c - 1)] = cid
            rec[f"hit_{c}"] = round(hit / max(1, look), 3)
            tot[c][0] += hit
            tot[c][1] += look
        out["top_reads"].append(rec)
    out["hit_rate"] = {c: round(h / max(1, n), 3) for c, (h, n) in tot.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

"""Extend profile of the seeding loop (oracle counts on the CPU): how many
bwt_extend calls per read produce a string of each length, and how many run on
size-1 intervals -- the numbers behind the k-mer interval table.

    python tools/ext_profile.py [--genome-mbp 3101.8] [--reads 20000] [--gpu]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--genome-mbp", type=float, default=3101.804739)
    p.add_argument("--reads", type=int, default=20000)
    p.add_argument("--gpu", action="store_true", help="build the index on the GPU")
    p.add_argument("--threads", type=int, default=16)
    p.add_argument("--out", default=None)
    a = p.parse_args()
    import smemgpu
    from smemgpu import synth
    from oracle import oracle
    t = time.time()
    g = synth.make_genome(int(a.genome_mbp * 1e6), seed=1, n_chrom=24)
    idx = smemgpu.Index.build_gpu(g.codes) if a.gpu else smemgpu.Index.build(g.codes)
    print(f"index {time.time() - t:.1f} s", flush=True)
    oi = oracle.OracleIndex(words=idx.words, primary=idx.primary, L2=idx.L2)
    rep = {"genome_mbp": a.genome_mbp, "reads": a.reads, "cases": {}}
    for name, rl, sub, opt in (("150bp_2pct", 150, 0.02, {}), ("150bp_5pct", 150, 0.05, {}),
                               ("250bp_2pct", 250, 0.02, {})):
        r = synth.make_reads(g.codes, a.reads, rl, seed=2, sub_rate=sub, n_rate=0.001)
        _, _, st = oracle.seed(oi, r.codes, r.offs, threads=a.threads, **opt)
        n = r.n
        hist = np.array(st.pop("n_ext_len"), dtype=np.float64) / n
        cum = np.cumsum(hist)
        d = {k: round(v / n, 2) for k, v in st.items()}
        d["ext_len_hist"] = [round(x, 2) for x in hist]
        d["frac_ext_len_le"] = {k: round(float(cum[k] / cum[-1]), 4) for k in range(8, 33)}
        rep["cases"][name] = d
        print(name, json.dumps(d), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(rep, fh, indent=1)
    oi.close()


if __name__ == "__main__":
    main()

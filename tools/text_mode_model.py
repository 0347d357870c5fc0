"""Model of a unique-interval text mode for the seeding loop (VERDICT round 5,
item 1), counted by the restatement on the bench's own reads.

An interval of size 1 keeps x[0] under forward extension and x[1] under
backward extension (software/bwt.c:416-429: the extension of a single row), so
whether it survives the next base is decided by the reference text alone: the
base after (forward) or before (backward) its one occurrence.  The text mode
this models replaces every Occ64 bucket load of such an extend by
  - one SA load per run of text compares (the occurrence's position; a full
    SA resident, 5 B per row, 31 GB at human size),
  - the 16-B .pac block of each 64 bases compared,
  - one ISA load whenever a text-compared interval is pushed (forward: its
    exact x[1]) or emitted as a SMEM (backward: its exact x[0]) -- a full ISA
    resident, another 31 GB,
which is the cheapest form of the mode (the verdict's variant with the dense
every-4th-row SA and an ISA sample adds <= 3 LF steps, one bucket load each, to
every SA and ISA load).  Counted per read (oracle/smem_oracle.c n_tm_*):
loads now = the Occ64 bucket loads of every used extend (n_bkt64, what
seed_wp_kernel issues), loads with the mode = loads now - n_tm_saved + n_tm_sa
+ n_tm_isa + text blocks, text blocks = runs + (bases - runs) / 64.

    python tools/text_mode_model.py [--genome-mbp 3101.8 --gpu] [--reads 20000] [--out f.json]
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)


def model(st: dict, n: int) -> dict:
    pr = {k: st[k] / n for k in ("n_ext", "n_bkt64", "n_ext_fwd", "n_ext_u1_fwd", "n_ext_u1_bwd", "n_tm_saved",
                                  "n_tm_sa", "n_tm_isa", "n_tm_runs", "n_tm_bases")}
    text_blocks = pr["n_tm_runs"] + max(0.0, pr["n_tm_bases"] - pr["n_tm_runs"]) / 64
    added = pr["n_tm_sa"] + pr["n_tm_isa"] + text_blocks
    after = pr["n_bkt64"] - pr["n_tm_saved"] + added
    # the LF-walk variant: <= 3 bucket loads per SA / ISA load (every-4th-row SA, every-4th-position
    # ISA sample: 1.5 LF steps on average each)
    after_lf = after + 1.5 * (pr["n_tm_sa"] + pr["n_tm_isa"])
    return {"per_read": {k: round(v, 2) for k, v in pr.items()},
            "text_blocks_per_read": round(text_blocks, 2),
            "loads_now": round(pr["n_bkt64"], 1),
            "loads_text_mode_full_sa_isa": round(after, 1),
            "loads_text_mode_lf_samples": round(after_lf, 1),
            "reduction_full_sa_isa": round(1 - after / pr["n_bkt64"], 4),
            "reduction_lf_samples": round(1 - after_lf / pr["n_bkt64"], 4),
            "u1_share_of_extends": round((pr["n_ext_u1_fwd"] + pr["n_ext_u1_bwd"]) / pr["n_ext"], 4),
            "forward_u1_extends_per_read": round(pr["n_ext_u1_fwd"], 1)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--genome-mbp", type=float, default=100.0)
    p.add_argument("--genome-profile", default="human", choices=("human", "uniform"))
    p.add_argument("--reads", type=int, default=20000)
    p.add_argument("--gpu", action="store_true", help="build the index on the GPU (human size)")
    p.add_argument("--threads", type=int, default=16)
    p.add_argument("--out", default=None)
    p.add_argument("--cache", default=os.path.join(tempfile.gettempdir(), "smem_bench_cache"))
    a = p.parse_args()
    import numpy as np
    import smemgpu
    from smemgpu import synth
    from oracle import oracle
    t = time.time()
    n_bp = int(a.genome_mbp * 1e6)
    # bench.py's cached genome + index (same seed and profile) when a bench ran before on this host
    base = os.path.join(a.cache, f"genome_{n_bp}_1{'_human' if a.genome_profile == 'human' else ''}")
    if os.path.exists(base + ".bwt") and os.path.exists(base + ".codes"):
        codes = np.memmap(base + ".codes", dtype=np.uint8, mode="r")
        idx = smemgpu.Index.read(base + ".bwt")
        print(f"bench cache {base}", flush=True)
    else:
        g = (synth.make_genome_human_like(n_bp, seed=1, n_chrom=24) if a.genome_profile == "human"
             else synth.make_genome(n_bp, seed=1, n_chrom=24))
        codes = g.codes
        idx = smemgpu.Index.build_gpu(codes) if a.gpu else smemgpu.Index.build(codes)
    print(f"index {time.time() - t:.1f} s", flush=True)
    oi = oracle.OracleIndex(words=idx.words, primary=idx.primary, L2=idx.L2)
    rep = {"genome_mbp": a.genome_mbp, "genome_profile": a.genome_profile, "reads": a.reads,
           "threshold": "build only if >= 25 % fewer loads per read (VERDICT round 5)", "cases": {}}
    for name, rl, sub, opt in (("c2_150bp_2pct", 150, 0.02, {}), ("c5_150bp_5pct", 150, 0.05, {}),
                               ("c4_250bp_2pct_k19", 250, 0.02, {})):
        r = synth.make_reads(np.asarray(codes), a.reads, rl, seed=2, sub_rate=sub, n_rate=0.001)
        _, _, st = oracle.seed(oi, r.codes, r.offs, threads=a.threads, **opt)
        d = model(st, r.n)
        rep["cases"][name] = d
        print(name, json.dumps(d), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(rep, fh, indent=1)
    oi.close()


if __name__ == "__main__":
    main()

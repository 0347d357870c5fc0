"""Backward-step shape of the seeding loop, from the restatement's counters.

Sizes the wave-parallel seeding kernel: how many entries a
backward step extends (software/bwt.c:812-826: every surviving interval of
`prev` with the same base), and how many of those extends read a list entry
at index >= NL (outside the per-owner LDS list).  Builds a synthetic genome
with the host builder, seeds reads with the oracle (test infrastructure, not
the product) and prints the histograms as JSON.

  python tools/wp_stats.py --mbp 100 --reads 20000 --nl 8 10 11 12 16
"""
import argparse
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mbp", type=float, default=100)
    ap.add_argument("--profile", default="uniform", choices=["uniform", "human"])
    ap.add_argument("--reads", type=int, default=20000)
    ap.add_argument("--len", type=int, default=150)
    ap.add_argument("--sub", type=float, default=0.02)
    ap.add_argument("--nl", type=int, nargs="+", default=[8, 10, 11, 12, 16])
    ap.add_argument("--cache", default="/tmp/wp_stats_idx")
    a = ap.parse_args()
    n_bp = int(a.mbp * 1e6)
    g = (synth.make_genome_human_like(n_bp, seed=1) if a.profile == "human" else synth.make_genome(n_bp, seed=1))
    os.makedirs(a.cache, exist_ok=True)
    fn = os.path.join(a.cache, f"{a.profile}_{n_bp}.bwt")
    if not os.path.exists(fn):
        idx = smemgpu.Index.build(g.codes)
        idx.write(fn)
        idx.close()
    oi = oracle.OracleIndex(fn)
    r = synth.make_reads(g.codes, a.reads, a.len, seed=7, sub_rate=a.sub)
    out = {"mbp": a.mbp, "profile": a.profile, "reads": a.reads, "len": a.len, "sub": a.sub, "by_nl": {}}
    for nl in a.nl:
        os.environ["ORC_LIST_LDS"] = str(nl)
        # the oracle reads ORC_LIST_LDS once per process: one child per NL
        import subprocess
        code = (f"import sys,json,os; sys.path[:0]={sys.path[:2]!r}; from oracle import oracle; "
                f"from smemgpu import synth; import numpy as np; "
                f"oi=oracle.OracleIndex({fn!r}); g=None; "
                f"d=np.load('/tmp/wp_stats_reads.npz'); "
                f"per,st=oracle.seed_stats(oi,d['codes'],d['offs'],threads=8); print(json.dumps(st))")
        np.savez("/tmp/wp_stats_reads.npz", codes=r.codes, offs=r.offs)
        res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=dict(os.environ),
                             check=True)
        st = json.loads(res.stdout.strip().splitlines()[-1])
        bwd = st["n_ext"] - st["n_ext_fwd"]
        out["by_nl"][nl] = {"bwd_task_hi_frac": st["n_bwd_task_hi"] / max(1, bwd),
                            "fwd_spill_per_read": st["n_fwd_spill"] / a.reads,
                            "bwd_push_hi_per_read": st["n_bwd_push_hi"] / a.reads}
        out["ext_per_read"] = st["n_ext"] / a.reads
        out["fwd_ext_per_read"] = st["n_ext_fwd"] / a.reads
        out["bwd_steps_per_read"] = st["n_bwd_step"] / a.reads
        out["bwd_ext_per_step"] = bwd / max(1, st["n_bwd_step"])
        out["fwd_push_per_read"] = st["n_fwd_push"] / a.reads
        out["smem1_per_read"] = st["n_smem1"] / a.reads
        h = np.array(st["n_step_hist"], dtype=float)
        out["step_hist_frac"] = (h / max(1.0, h.sum())).round(4).tolist()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

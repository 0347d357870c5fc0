"""A/B of the ksw_extend2 kernels on problems shaped like mem_chain2aln's
extensions (synth.make_ksw_tasks over a synthetic genome): one problem per
wave (the default), four per wave (SMEM_KSW_G16), one per lane (SMEM_KSW_LANE),
the lane kernel also on the problems sorted by query length.  Every variant's
results must equal the default's.

    python tools/ksw_ab.py [--problems 200000] [--reps 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--problems", type=int, default=200000)
    p.add_argument("--unique", type=int, default=20000)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--max-qlen", type=int, default=0, help="keep only problems with qlen <= this (0: all)")
    p.add_argument("--only", default="", help="variant names to run, joined by , or + (default: all)")
    a = p.parse_args()
    import smemgpu
    from smemgpu import synth
    g = synth.make_genome(2_000_000, seed=771, n_chrom=1)
    idx = smemgpu.Index.build(g.codes)
    gpu = smemgpu.Gpu(idx, device=0)
    kb = synth.make_ksw_tasks(g.codes, a.unique, seed=771)
    if a.max_qlen:
        kb = synth.KswBatch(kb.tasks[kb.tasks["qlen"] <= a.max_qlen], kb.q, kb.t, kb.mat)
    tile = max(1, a.problems // a.unique)
    big = synth.KswBatch(np.tile(kb.tasks, tile), kb.q, kb.t, kb.mat)
    order = np.argsort(big.tasks["qlen"], kind="stable")
    srt = synth.KswBatch(big.tasks[order], kb.q, kb.t, kb.mat)
    ql = big.tasks["qlen"]
    from oracle import oracle
    oracle.dp_cells(True)
    oracle.ksw(kb)
    cells = oracle.dp_cells(True)[0] * tile
    print(f"{big.tasks.size} problems, qlen mean {ql.mean():.1f} max {ql.max()}, {cells / big.tasks.size:.0f} in-band "
          "cells each", flush=True)
    ref = None
    for name, env, batch in [("wave", {"SMEM_KSW_LANE": "0"}, big), ("g16", {"SMEM_KSW_G16": "1"}, big),
                             ("lane", {"SMEM_KSW_LANE": "1"}, big), ("lane_sorted", {"SMEM_KSW_LANE": "1"}, srt),
                             ("wave_sorted", {"SMEM_KSW_LANE": "0"}, srt)]:
        if a.only and name not in a.only.replace("+", ",").split(","):
            continue
        os.environ.pop("SMEM_KSW_G16", None)
        os.environ.pop("SMEM_KSW_LANE", None)
        os.environ.update(env)
        best = None
        for _ in range(a.reps):
            got, ms = gpu.ksw_extend(batch)
            best = ms if best is None else min(best, ms)
        if batch is srt:
            un = np.empty_like(got)
            un[order] = got
            got = un
        if ref is None:
            ref = got
        same = bool(np.array_equal(got, ref))
        print(f"{name:12s} {best:8.3f} ms  {big.tasks.size / best / 1e3:8.2f} M problems/s  "
              f"{cells / best / 1e6:8.1f} GCUPS  same={same}", flush=True)
    gpu.close()


if __name__ == "__main__":
    main()

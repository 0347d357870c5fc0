"""The seeding kernel's request ceiling on its own access stream (VERDICT
round 5, item 3): record every Occ64 bucket load the kernel makes for a sample
of the bench's reads (the restatement's trace, oracle.seed_trace, on the
bench's cached human-size index) and replay it with tools/replay_ceiling at the
kernel's occupancy, beside the same replay with the bucket indices hashed
uniformly (the random-gather ceiling at the same occupancy and chain shape).

    python tools/replay_ceiling.py [--genome-profile human] [--reads 200000] [--waves 12,15,16] [--out f.json]

Needs bench.py's cache of the index (run bench.py first in the same gpurun call)
and tools/replay_ceiling built (hipcc --offload-arch=gfx950 -O3 -o tools/bin/replay_ceiling
tools/replay_ceiling.hip).
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--genome-mbp", type=float, default=3101.804739)
    p.add_argument("--genome-profile", default="human", choices=("human", "uniform"))
    p.add_argument("--reads", type=int, default=200000)
    p.add_argument("--sub", type=float, default=0.02)
    p.add_argument("--waves", default="12,15,16")
    p.add_argument("--reps", type=int, default=4)
    p.add_argument("--threads", type=int, default=16)
    p.add_argument("--cache", default=os.path.join(tempfile.gettempdir(), "smem_bench_cache"))
    p.add_argument("--out", default=None)
    a = p.parse_args()
    import smemgpu
    from smemgpu import synth
    from oracle import oracle
    n_bp = int(a.genome_mbp * 1e6)
    base = os.path.join(a.cache, f"genome_{n_bp}_1{'_human' if a.genome_profile == 'human' else ''}")
    codes = np.memmap(base + ".codes", dtype=np.uint8, mode="r")
    idx = smemgpu.Index.read(base + ".bwt")
    oi = oracle.OracleIndex(words=idx.words, primary=idx.primary, L2=idx.L2)
    r = synth.make_reads(np.asarray(codes), a.reads, 150, seed=2, sub_rate=a.sub, n_rate=0.001)
    t = time.time()
    # the trace in chunks on a thread pool (orc_seed_trace is one thread each; ctypes drops the GIL)
    k = a.threads
    cuts = np.linspace(0, r.n, k + 1).astype(np.int64)

    def one(i):
        lo, hi = cuts[i], cuts[i + 1]
        offs = r.offs[lo:hi + 1] - r.offs[lo]
        return oracle.seed_trace(oi, r.codes[r.offs[lo]:r.offs[hi]], offs)
    with ThreadPoolExecutor(k) as ex:
        parts = list(ex.map(one, range(k)))
    loads = np.concatenate([pt[0] for pt in parts])
    roff = np.zeros(r.n + 1, np.uint64)
    o, at = 0, 0
    for (tr, ro) in parts:
        nr = ro.size - 1
        roff[at:at + nr] = ro[:nr] + o
        o += tr.size
        at += nr
    roff[r.n] = o
    print(f"trace: {r.n} reads, {loads.size} bucket loads ({loads.size / r.n:.1f} per read) in {time.time() - t:.1f} s",
          flush=True)
    n_buckets = (int(idx.L2[4]) + 63) // 64 + 1  # Occ64: one 32-B bucket per 64 symbols ($ row excluded)
    tf = os.path.join(tempfile.gettempdir(), "smem_replay_trace.bin")
    with open(tf, "wb") as fh:
        fh.write(np.array([r.n, loads.size], np.uint64).tobytes())
        fh.write(roff.tobytes())
        fh.write(loads.astype(np.uint32).tobytes())
    del loads
    exe = os.path.join(ROOT, "tools", "bin", "replay_ceiling")
    rep = {"reads": r.n, "genome_profile": a.genome_profile, "sub": a.sub, "n_buckets": n_buckets, "runs": []}
    for w in [int(x) for x in a.waves.split(",") if x]:
        for uni in (0, 1):
            out = subprocess.run(["timeout", "-k", "5", "120", exe, tf, str(n_buckets), str(w), str(a.reps), str(uni)],
                                 capture_output=True, text=True, check=True).stdout
            runs = [json.loads(x) for x in out.splitlines() if x.startswith("{")]
            best = max(runs, key=lambda x: x["Gbuckets_per_s"])
            rep["runs"].append(best)
            print(json.dumps(best), flush=True)
    os.remove(tf)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(rep, fh, indent=1)
    oi.close()


if __name__ == "__main__":
    main()

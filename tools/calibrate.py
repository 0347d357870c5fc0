"""Single-core calibration of the CPU restatement against the compiled
reference (SURVEY.md §8(d) "CPU baseline"): both seed the same synthetic
reads over the same index, one thread each, and the ratio is recorded in
profiles/calibration.json.  Runs on the CPU (this container or the box).

    python tools/calibrate.py [--genome-mbp 20 --reads 20000 --threads 1 8]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--genome-mbp", type=float, default=20.0)
    p.add_argument("--reads", type=int, default=20000)
    p.add_argument("--read-len", type=int, default=150)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--threads", type=int, nargs="+", default=[1, 8])
    p.add_argument("--out", default=os.path.join(ROOT, "profiles", "calibration.json"))
    a = p.parse_args()
    from oracle import oracle
    import smemgpu
    from smemgpu import synth
    oracle.build()
    if not oracle.ref_available():
        sys.exit("compiled reference (oracle/_ref) not built: /root/reference absent")
    g = synth.make_genome(int(a.genome_mbp * 1e6), seed=a.seed, n_chrom=4)
    reads = synth.make_reads(g.codes, a.reads, a.read_len, seed=a.seed + 17, sub_rate=0.02, n_rate=0.001)
    t = time.time()
    idx = smemgpu.Index.build(g.codes)
    build_s = time.time() - t
    rows = []
    with tempfile.TemporaryDirectory() as d:
        bwt, smrd = os.path.join(d, "g.bwt"), os.path.join(d, "r.smrd")
        idx.write(bwt)
        synth.write_smrd(smrd, reads)
        oi = oracle.OracleIndex(words=idx.words, primary=idx.primary, L2=idx.L2)
        for th in a.threads:
            best_port, best_ref = None, None
            for _ in range(3):
                s, _ = oracle.seed_timed(oi, reads.codes, reads.offs, threads=th)
                best_port = s if best_port is None else min(best_port, s)
                r = oracle.ref_bench(bwt, smrd, th, reads.n)["seconds"]
                best_ref = r if best_ref is None else min(best_ref, r)
            rows.append({"threads": th, "port_reads_per_s": round(reads.n / best_port, 1),
                         "reference_reads_per_s": round(reads.n / best_ref, 1),
                         "port_over_reference": round(best_ref / best_port, 3)})
        oi.close()
    out = {"what": "seeding loop (mem_insert_seed -> smem_next2 -> bwt_smem1), CPU restatement (oracle/smem_oracle.c) "
                   "vs the reference compiled from its own sources (oracle/_ref/ref_harness), same index and reads, "
                   "best of 3",
           "workload": {"genome_mbp": a.genome_mbp, "reads": a.reads, "read_len": a.read_len, "sub": 0.02,
                        "seed": a.seed},
           "index_build_s": round(build_s, 1), "host_cpus": os.cpu_count(), "rows": rows,
           "measured": time.strftime("%Y-%m-%d %H:%M:%S")}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

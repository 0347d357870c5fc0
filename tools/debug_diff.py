"""Print the first reads whose GPU lists differ from the oracle (debug aid)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)

import smemgpu  # noqa: E402
from smemgpu import synth  # noqa: E402
from oracle import oracle  # noqa: E402


def main():
    variant = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    genome = synth.make_genome(400_000, seed=21)
    idx = smemgpu.Index.build(genome.codes)
    reads = synth.make_reads(genome.codes, 2000, 150, seed=107)
    ref = oracle.OracleIndex(words=idx.words, primary=idx.primary, L2=idx.L2)
    want, _, _ = oracle.seed(ref, reads.codes, reads.offs)
    gpu = smemgpu.Gpu(idx, device=0, variant=variant)
    got = smemgpu.seed(gpu, reads.codes, reads.offs).to_smgo()
    a, b = synth.read_smgo(got), synth.read_smgo(want)
    bad = [i for i in range(len(b)) if len(a[i]) != len(b[i]) or any(
        x.shape != y.shape or (x != y).any() for x, y in zip(a[i], b[i]))]
    print(f"variant {variant}: {len(bad)} reads differ")
    for r in bad[:3]:
        print(f"--- read {r}: gpu {len(a[r])} lists, oracle {len(b[r])} lists; seq",
              "".join("ACGTN"[c] for c in reads.read(r)))
        for c in range(max(len(a[r]), len(b[r]))):
            ga = a[r][c] if c < len(a[r]) else None
            gb = b[r][c] if c < len(b[r]) else None
            fmt = lambda m: None if m is None else [(int(x[0]), int(x[1]), int(x[2]), int(x[3]) >> 32, int(x[3]) & 0xffffffff) for x in m]
            same = ga is not None and gb is not None and ga.shape == gb.shape and (ga == gb).all()
            print(f"  call {c} {'==' if same else '!='}")
            if not same:
                print("    gpu   ", fmt(ga))
                print("    oracle", fmt(gb))
    gpu.close()


if __name__ == "__main__":
    main()

"""Minimal workload for rocprofv3 counter passes: the bench's own index (same
cache) and the bench's own resident reads (bench.make_reads: same blocks,
seeds and options), seeded --launches times.  Meant to run under

    rocprofv3 --pmc <counters> --kernel-include-regex 'seed_(wp_)?kernel' -- python tools/prof_run.py [bench args]

Any bench.py argument selects the workload (--config, --genome-profile,
--reads, --genome-mbp ...); --launches is this tool's own (--variant / --kmer-k are bench's).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)


def main():
    import argparse
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument("--launches", type=int, default=1)
    p.add_argument("--stats-out", default=None, help="write the launch shape and library ids here (JSON)")
    own, rest = p.parse_known_args()
    import bench
    import smemgpu
    a = bench.parse(rest)
    idx, _, _, codes = bench.get_index(a, 0, lambda: None, 0)
    reads = bench.make_reads(a, 0, codes, 1)
    gpu = smemgpu.Gpu(idx, device=0, lanes_per_cu=a.lanes_per_cu, variant=a.variant, kmer_k=a.kmer_k)
    b = gpu.batch(reads.n, reads.codes.size, int(reads.lens.max()))
    b.set_reads(reads.codes, reads.offs)
    opt = smemgpu.Options(min_seed_len=a.min_seed_len)
    for _ in range(own.launches):
        t = time.time()
        b.run(opt)
        print(f"launch: kernel {b.stats()['kernel_ms']:.3f} ms, wall {1e3 * (time.time() - t):.1f} ms", flush=True)
    if own.stats_out:
        import json
        st = b.stats()
        with open(own.stats_out, "w") as fh:
            json.dump({"grid": st["grid"], "block": st["block"], "build_id": smemgpu.build_id(),
                       "kernel_id": smemgpu.kernel_id(), "variant": gpu.variant}, fh)
    b.close()
    gpu.close()


if __name__ == "__main__":
    main()

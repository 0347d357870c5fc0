"""The seeding kernel's per-read raw-output capacity (smem_gpu_set_intv_cap)
against the reads that overflow it (and take the overflow pass) and the
launch time, on the bench's reads: what a worker slot's largest buffer
(d_out_intv, 32 B per slot) can be cut to.

    python tools/intv_cap_sweep.py [--caps 48,56,64,80,0] [bench args]   (0: the default, max_len / 2 + 32)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)


def main():
    import argparse
    import json
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument("--caps", default="48,56,64,80,0")
    p.add_argument("--reps", type=int, default=3)
    own, rest = p.parse_known_args()
    import torch
    torch.cuda.device_count()
    import bench
    import smemgpu
    a = bench.parse(rest)
    idx, _, sa, codes = bench.get_index(a, 0, lambda: None, 0)
    reads = bench.make_reads(a, 0, codes, 1)
    for cap in [int(x) for x in own.caps.split(",")]:
        gpu = smemgpu.Gpu(idx, device=0, intv_cap=cap)
        b = gpu.batch(reads.n, reads.codes.size, int(reads.lens.max()))
        b.set_reads(reads.codes, reads.offs)
        opt = smemgpu.Options(min_seed_len=a.min_seed_len)
        ms = []
        for _ in range(own.reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            b.run(opt)
            ms.append((time.perf_counter() - t) * 1e3)
        st = b.stats()
        print(json.dumps({"cap": cap or "default", "reads": reads.n, "overflow_reads": st.get("n_overflow"),
                          "run_ms": [round(x, 2) for x in ms], "kernel_ms": st.get("kernel_ms"),
                          "n_intv": st.get("n_intv")}), flush=True)
        b.close()
        gpu.close()


if __name__ == "__main__":
    main()

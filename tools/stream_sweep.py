"""Sweep the streaming path (smem_gpu_seed_stream) over chunk sizes and
worker counts on one read set, beside the raw pinned D2H / H2D copy rates.

    python tools/stream_sweep.py [bench args, e.g. --config c5] [--chunks 262144,524288] [--workers 3,4,6]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)


def copy_rates():
    import torch
    n = 1 << 30
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    dv = torch.empty(n, dtype=torch.uint8, device="cuda")
    out = {}
    for name, f in (("h2d", lambda: dv.copy_(h, non_blocking=True)), ("d2h", lambda: h.copy_(dv, non_blocking=True))):
        f()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        out[name + "_GBps"] = round(5 * n / (time.perf_counter() - t) / 1e9, 2)
    return out


def main():
    import argparse
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument("--chunks", default="262144,524288")
    p.add_argument("--workers", default="3,4,6")
    p.add_argument("--packed", default="1")
    own, rest = p.parse_known_args()
    import torch
    torch.cuda.device_count()   # as bench.py's Dist does, before libsmemgpu touches the device
    import bench
    import smemgpu
    a = bench.parse(rest)
    idx, _, sa, codes = bench.get_index(a, 0, lambda: None, 0)
    t = time.time()
    n = a.stream_reads or a.reads
    reads = bench.make_reads(a, 0, codes, 1, n, salt=1)
    # libsmemgpu's HIP runtime must initialise the device before torch's
    # (bench.py has the same order)
    gpu = smemgpu.Gpu(idx, device=0)
    print(json.dumps({"reads": reads.n, "gen_s": round(time.time() - t, 1), **copy_rates()}), flush=True)
    opt = smemgpu.Options(min_seed_len=a.min_seed_len)
    b = gpu.batch(1 << 20, (1 << 20) * a.read_len, a.read_len)
    sub = reads.subset(range(1 << 20)) if reads.n > (1 << 20) else reads
    b.set_reads(sub.codes, sub.offs)
    b.run(opt)
    b.run(opt)
    st = b.stats()
    b.close()
    print(json.dumps({"resident_1M_kernel_ms": st["kernel_ms"], "compact_ms": st["compact_ms"]}), flush=True)
    for pk in (bool(int(x)) for x in own.packed.split(",")):
      for c in (int(x) for x in own.chunks.split(",")):
        for w in (int(x) for x in own.workers.split(",")):
            warm = reads.subset(range(min(reads.n, c * w)))
            gpu.seed_stream(warm.codes, warm.offs, opt, chunk_reads=c, workers=w, pairs=a.pairs, packed=pk)
            s, _ = gpu.seed_stream(reads.codes, reads.offs, opt, chunk_reads=c, workers=w, pairs=a.pairs, packed=pk)
            print(json.dumps({"packed": pk, "chunk": c, "workers": w, "reads_per_s": round(s["n_reads"] / s["wall_s"], 1),
                              "wall_s": round(s["wall_s"], 3), "d2h_GB": round(s["d2h_bytes"] / 1e9, 2),
                              "d2h_GBps_eff": round(s["d2h_bytes"] / s["wall_s"] / 1e9, 1),
                              "stage_s": round(s["stage_s"], 3), "run_s": round(s["run_s"], 3),
                              "fetch_s": round(s["fetch_s"], 3)}), flush=True)
    gpu.close()


if __name__ == "__main__":
    main()

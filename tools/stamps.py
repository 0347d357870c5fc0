"""Per-wave cycle split of the seeding kernel (stamped diagnostic variant 9).
Shares only: the stamps themselves perturb the schedule."""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)


PHASES = ["BWD_RES", "BWD_J", "FWD_RES", "FWD", "FWD_DONE", "BWD_STEP", "SMEM_END", "OVF", "NEXT2", "SMEM_BEGIN",
          "FETCH"]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--genome-mbp", type=float, default=1000)
    p.add_argument("--reads", type=int, default=1_000_000)
    p.add_argument("--lanes-per-cu", type=int, default=0)
    p.add_argument("--variant", type=int, default=2, help="production variant timed beside the stamped one")
    p.add_argument("--cache", default=os.path.join(tempfile.gettempdir(), "smem_bench_cache"))
    a = p.parse_args()
    import smemgpu
    from smemgpu import synth
    os.makedirs(a.cache, exist_ok=True)
    n_bp = int(a.genome_mbp * 1e6)
    key = os.path.join(a.cache, f"genome_{n_bp}_1.bwt")
    g = synth.make_genome(n_bp, seed=1, n_chrom=24)
    if not os.path.exists(key):
        smemgpu.Index.build_gpu(g.codes).write(key)
    idx = smemgpu.Index.read(key)
    reads = synth.make_reads(g.codes, a.reads, 150, seed=1000 + 7919, sub_rate=0.02, n_rate=0.001)
    for variant in (a.variant, 9):
        gpu = smemgpu.Gpu(idx, device=0, lanes_per_cu=a.lanes_per_cu, variant=variant)
        b = gpu.batch(reads.n, reads.codes.size, int(reads.lens.max()))
        b.set_reads(reads.codes, reads.offs)
        b.run()
        b.run()
        st = b.stats()
        print(f"variant {variant}: kernel {st['kernel_ms']:.2f} ms", flush=True)
        if variant == 9:
            w = b.debug_words(st["grid"] * 4 * 32).reshape(-1, 32).astype(np.float64)
            adv, fet, comp, it, act, t0, t1 = (w[:, k] for k in range(7))
            tot = adv.sum() + fet.sum() + comp.sum()
            out = {
                "waves": int(w.shape[0]),
                "iters_per_wave_mean": float(it.mean()),
                "active_lanes_per_iter": float(act.sum() / it.sum()),
                "cycles_per_iter_adv": float(adv.sum() / it.sum()),
                "cycles_per_iter_fetch": float(fet.sum() / it.sum()),
                "cycles_per_iter_comp": float(comp.sum() / it.sum()),
                # t0 / t1: s_memrealtime (100 MHz, chip-wide) -> ms from the first wave start
                "wave_start_spread_ms": float((t0.max() - t0.min()) * 1e-5),
                "wave_end_ms_p10_p50_p90_max": [float(np.percentile(t1 - t0.min(), q) * 1e-5) for q in (10, 50, 90, 100)],
                "waves_alive_at_ms": {f"{m:g}": int(((t1 - t0.min()) * 1e-5 > m).sum())
                                      for m in np.linspace(0, float((t1 - t0.min()).max() * 1e-5), 11)},
                "passes_per_iter": float(w[:, 23].sum() / it.sum()),
                "block_execs_per_iter": {n: round(float(w[:, 8 + k].sum() / it.sum()), 3) for k, n in enumerate(PHASES)},
                "share_adv_fetch_comp": [float(adv.sum() / tot), float(fet.sum() / tot), float(comp.sum() / tot)],
            }
            print(json.dumps(out, indent=1), flush=True)
        b.close()
        gpu.close()


if __name__ == "__main__":
    main()

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
    """Any bench.py argument selects the workload (--genome-profile, --config,
    --reads ...: the bench's own cached index and reads); --compare is the
    production variant timed beside the stamped one, --out a JSON file."""
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument("--compare", type=int, default=2, help="production variant timed beside the stamped one")
    p.add_argument("--stamped", type=int, default=9, help="the stamped variant (9: default kernel, 25: the PFCH variant 24)")
    p.add_argument("--out", default=None)
    own, rest = p.parse_known_args()
    import bench
    import smemgpu
    a = bench.parse(rest)
    idx, _, _, codes = bench.get_index(a, 0, lambda: None, 0)
    reads = bench.make_reads(a, 0, codes, 1)
    a.variant = own.compare
    results = {"workload": {"genome_profile": a.genome_profile, "genome_mbp": a.genome_mbp, "reads": reads.n,
                            "read_len": a.read_len, "sub": a.sub}}
    for variant in (a.variant, own.stamped):
        gpu = smemgpu.Gpu(idx, device=0, lanes_per_cu=a.lanes_per_cu, variant=variant)
        opt = smemgpu.Options(min_seed_len=a.min_seed_len)
        b = gpu.batch(reads.n, reads.codes.size, int(reads.lens.max()))
        b.set_reads(reads.codes, reads.offs)
        b.run(opt)
        b.run(opt)
        st = b.stats()
        print(f"variant {variant}: kernel {st['kernel_ms']:.2f} ms", flush=True)
        results[f"kernel_ms_variant_{variant}"] = st["kernel_ms"]
        if variant == own.stamped:
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
            results["stamps"] = out
        b.close()
        gpu.close()
    if own.out:
        with open(own.out, "w") as fh:
            json.dump(results, fh, indent=1)


if __name__ == "__main__":
    main()

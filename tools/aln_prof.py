"""Alignment-stage workload for rocprofv3 (kernel trace or counter passes):
the bench's index, reads and options, then seeding + SA + chaining once and
smem_batch_chain2aln --launches times.

    rocprofv3 --pmc <counters> --kernel-include-regex aln_kernel -- python tools/aln_prof.py [bench args]
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
    p.add_argument("--launches", type=int, default=2)
    p.add_argument("--cycles", default=None, help="write per-read shader cycles of the last launch here (u64)")
    p.add_argument("--lib", default=None, help="another libsmemgpu build (diagnostics)")
    p.add_argument("--compare", action="store_true", help="fetch the regions after each setting: all settings must "
                   "give the same bytes (e.g. SMEM_ALN_LANE=0 / 1)")
    p.add_argument("--env-sweep", default="", help="';'- (or '/'-) separated settings, each ','-separated VAR=value: "
                   "--launches launches under each, in turn (the library reads them per call)")
    own, rest = p.parse_known_args()
    import torch
    torch.cuda.device_count()  # as bench.py's Dist does, before libsmemgpu touches the device
    import bench
    import smemgpu
    if own.lib:
        smemgpu.lib.LIB_PATH = os.path.abspath(own.lib)
    from oracle import oracle
    a = bench.parse(rest)
    idx, _, sa, codes = bench.get_index(a, 0, lambda: None, 0)
    reads = bench.make_reads(a, 0, codes, 1)
    gpu = smemgpu.Gpu(idx, device=0, lanes_per_cu=a.lanes_per_cu, variant=a.variant, kmer_k=a.kmer_k)
    gpu.load_sa(sa)
    gpu.load_pac(bench.pack_pac(codes), idx.seq_len // 2)
    b = gpu.batch(reads.n, reads.codes.size, int(reads.lens.max()))
    b.set_reads(reads.codes, reads.offs)
    opt = smemgpu.Options(min_seed_len=a.min_seed_len)
    b.run(opt)
    b.sa(opt.min_seed_len, 10000)
    b.chain(idx.seq_len // 2)
    settings = [s for s in own.env_sweep.replace("/", ";").split(";") if s] or [""]
    first = None
    for setting in settings:
        kv = dict(x.split("=", 1) for x in setting.replace("+", ",").split(",") if x)
        saved = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        for k in range(own.launches):
            if own.cycles and k == own.launches - 1:
                os.environ["SMEM_ALN_CYCLES"] = own.cycles
            t = time.time()
            b.chain2aln(oracle.aln_opt(min_seed_len=opt.min_seed_len))
            st = b.stats()
            print(f"chain2aln{' [' + setting + ']' if setting else ''}: {st['aln_ms']:.3f} ms, {st['n_regs']} regions, "
                  f"{st['n_chains']} chains, wall {1e3 * (time.time() - t):.1f} ms", flush=True)
        if own.compare:
            import numpy as np
            res = b.fetch(8)  # FETCH_REGS
            regs = (res.regs.copy(), np.asarray(res.reg_off).copy())
            if first is None:
                first = regs
            same = regs[0].size == first[0].size and bool((regs[0] == first[0]).all()) and \
                bool((regs[1] == first[1]).all())
            print(f"regions [{setting}] {regs[0].size // 64}: {'same as' if same else 'DIFFER from'} the first setting's",
                  flush=True)
            if not same:
                raise SystemExit(1)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    if own.cycles:  # the slowest reads' cycles, walk split and chain / seed counts (small enough to copy back)
        import json
        import numpy as np
        res = b.fetch()
        cyc = np.fromfile(own.cycles, dtype=np.uint64).astype(np.int64)
        walk = np.fromfile(own.cycles + ".walk", dtype=np.uint64).astype(np.int64).reshape(-1, 4)
        off = np.asarray(res.chain_off, dtype=np.int64)
        cn = np.asarray(res.chains["n"], dtype=np.int64)
        top = []
        for r in np.argsort(-cyc)[:30]:
            ns = cn[off[r]:off[r + 1]]
            top.append(dict(read=int(r), cycles=int(cyc[r]), ms_at_2_4ghz=round(cyc[r] / 2.4e6, 3),
                            chains=int(ns.size), seeds=int(ns.sum()), chains_over_64=int((ns > 64).sum()),
                            max_chain=int(ns.max()) if ns.size else 0,
                            walk_full_cycles=int(walk[r, 0]), walk_hash_cycles=int(walk[r, 1]),
                            walk_big_chains=int(walk[r, 2] & 0xFFFFFFFF), walk_big_seeds=int(walk[r, 2] >> 32),
                            walk_hops=int(walk[r, 3])))
        with open(own.cycles + ".top.json", "w") as fh:
            json.dump(top, fh, indent=1)
        os.unlink(own.cycles)
        os.unlink(own.cycles + ".walk")
    b.close()
    gpu.close()


if __name__ == "__main__":
    main()

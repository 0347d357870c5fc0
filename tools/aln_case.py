"""One golden chain2aln case through a given libsmemgpu build (bisecting
helper): python tools/aln_case.py --lib <so> [--fix g1_default_std]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lib", default=None)
    p.add_argument("--fix", default="g1_default_std")
    a = p.parse_args()
    import smemgpu
    from smemgpu import lib
    if a.lib:
        lib.LIB_PATH = os.path.abspath(a.lib)
    from oracle import oracle
    from tests import golden_data
    from tests import test_aln as T
    fix = [f for f in T.FIX if f["file"].split(".")[0] == a.fix][0]
    reads, chains, chain_off, seeds = T._case_inputs(fix)
    want, want_off = golden_data.smrg_parse(golden_data.smrg(fix))
    idx = smemgpu.Index.read(golden_data.files(fix["genome"], T._tmpdir())["bwt"])
    gpu = smemgpu.Gpu(idx, device=0)
    t = time.time()
    raw, off, ms = gpu.chain2aln(golden_data.pac(fix["genome"]), golden_data.l_pac(fix["genome"]), reads.codes,
                                 reads.offs, chains, chain_off, seeds,
                                 oracle.aln_opt(w=fix["w"], min_seed_len=fix["min_seed_len"]))
    got = np.frombuffer(raw.tobytes(), dtype=golden_data.ALNREG_DT)
    T._assert_same(got, off, want, want_off)
    print(f"{a.fix} ok: {ms:.2f} ms kernel, {time.time() - t:.2f} s", flush=True)
    gpu.close()


if __name__ == "__main__":
    main()

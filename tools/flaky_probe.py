"""Repeat `bwa-gpu mem` on a golden read set under several settings and count
the runs whose SAM differs from the reference's golden SAM (or that crash):
a probe for an intermittent multi-context failure (round 6).

    python tools/flaky_probe.py --reps 6 --out gpurun_out/flaky.json
"""
import argparse
import gzip
import json
import os
import shutil
import subprocess
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BWA = os.path.join(ROOT, "oracle", "_ref", "bwa-gpu")
GOLD = os.path.join(ROOT, "tests", "golden")

SETTINGS = {
    "ctx8_t16_b37": (16, 37, {"SMEM_GPU_DEVICES": ",".join(["0"] * 8)}),
    "ctx8_t16_b37_stages1": (16, 37, {"SMEM_GPU_DEVICES": ",".join(["0"] * 8), "SMEM_GPU_STAGES": "1"}),
    "ctx8_t16_b37_nooverlap": (16, 37, {"SMEM_GPU_DEVICES": ",".join(["0"] * 8), "SMEM_GPU_OVERLAP": "0"}),
    "ctx1_t16_b37": (16, 37, {"SMEM_GPU_DEVICES": "0"}),
    "ctx8_t8_b37": (8, 37, {"SMEM_GPU_DEVICES": ",".join(["0"] * 8)}),
    "ctx8_t16_b37_syncinit": (16, 37, {"SMEM_GPU_DEVICES": ",".join(["0"] * 8), "SMEM_GPU_SYNC_INIT": "1"}),
    "ctx8_t16_b37_walk": (16, 37, {"SMEM_GPU_DEVICES": ",".join(["0"] * 8), "SMEM_GPU_DENSIFY": "walk"}),
    "ctx8_t16_b37_saraw": (16, 37, {"SMEM_GPU_DEVICES": ",".join(["0"] * 8), "SMEM_GPU_SA_RAW": "1"}),
    "ctx2_t16_b37": (16, 37, {"SMEM_GPU_DEVICES": "0,0"}),
    "ctx8_t16_b37_guard": (16, 37, {"SMEM_GPU_DEVICES": ",".join(["0"] * 8), "SMEM_GPU_GUARD": "1"}),
    "ctx8_t16_b37_pool_check": (16, 37, {"SMEM_GPU_DEVICES": ",".join(["0"] * 8), "SMEM_GPU_DENSIFY_POOL": "1",
                                         "SMEM_GPU_SA_CHECK": "1"}),
    "ctx8_t16_b37_check": (16, 37, {"SMEM_GPU_DEVICES": ",".join(["0"] * 8), "SMEM_GPU_SA_CHECK": "1"}),
    "ctx1_t16_b37_guard": (16, 37, {"SMEM_GPU_DEVICES": "0", "SMEM_GPU_GUARD": "1"}),
    "ctx8_t8_b37_guard": (8, 37, {"SMEM_GPU_DEVICES": ",".join(["0"] * 8), "SMEM_GPU_GUARD": "1"}),
    "ctx1_t1_b37_guard": (1, 37, {"SMEM_GPU_DEVICES": "0", "SMEM_GPU_GUARD": "1"}),
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=6)
    p.add_argument("--settings", default=",".join(SETTINGS))
    p.add_argument("--g", default="g1")
    p.add_argument("--kind", default="se")
    p.add_argument("--out", default=None)
    p.add_argument("--bwa", default=BWA, help="another build (e.g. oracle/_ref/bwa-gpu-asan: make -C integration ASAN=1)")
    a = p.parse_args()
    d = tempfile.mkdtemp()
    fa = os.path.join(d, f"{a.g}.fa")
    with gzip.open(os.path.join(GOLD, f"{a.g}.fa.gz"), "rb") as src, open(fa, "wb") as dst:
        shutil.copyfileobj(src, dst)
    subprocess.run([BWA, "index", "-a", "is", fa], check=True, capture_output=True, cwd=d,
                   env=dict(os.environ, SMEM_GPU_INDEX="0"))
    with gzip.open(os.path.join(GOLD, "sam", f"{a.g}_{a.kind}.sam.gz"), "rt") as fh:
        want = [l for l in fh.read().split("\n") if l and not l.startswith("@PG")]
    fq = os.path.join(GOLD, "sam", f"{a.g}_{a.kind}.fq.gz")
    rep = {}
    for name in a.settings.split(","):
        t, b, env = SETTINGS[name]
        res = []
        for k in range(a.reps):
            args = [a.bwa, "mem", "-t", str(t), "-b", str(b)] + (["-p"] if a.kind == "pe" else []) + [fa, fq]
            t0 = time.time()
            pr = subprocess.run(args, capture_output=True, text=True, timeout=300,
                                env=dict(os.environ, SMEM_GPU_CRASH_TRACE="0" if "asan" in a.bwa else "1",
                                         ASAN_OPTIONS="detect_leaks=0", **env))
            got = [l for l in pr.stdout.split("\n") if l and not l.startswith("@PG")]
            diff = [i for i, (x, y) in enumerate(zip(got, want)) if x != y]
            r = {"rc": pr.returncode, "lines": len(got), "diff": len(diff) + abs(len(got) - len(want)),
                 "s": round(time.time() - t0, 2)}
            if diff:
                r["first"] = [got[diff[0]][:300], want[diff[0]][:300]]
            gl = [l for l in pr.stderr.split("\n") if l.startswith("[smem guard]") or
                  (l.startswith("[M::sa_check]") and " 0 of " not in l)]
            hs = sorted(set(l.split("dense hash ")[1][:16] for l in pr.stderr.split("\n") if "dense hash " in l))
            if hs:
                r["sa_hashes"] = hs
            if gl:
                r["guard"] = gl[:20]
            if pr.returncode:
                c = pr.stderr.find("[smem crash]")
                c = pr.stderr.find("ERROR: AddressSanitizer") if c < 0 else c
                r["err"] = pr.stderr[c:c + 6000] if c >= 0 else pr.stderr[-1500:]
            res.append(r)
            print(name, k, json.dumps(r)[:600], flush=True)
        rep[name] = res
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(rep, fh, indent=1)


if __name__ == "__main__":
    main()

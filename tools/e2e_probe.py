"""Run the product path (bwa-gpu mem) on the bench's human-size index and reads
with the stderr kept: per-batch GPU timings, refusals and their error text.

    python tools/e2e_probe.py [--reads 200000] [--threads 16] [--legs gpu/ref] [bench args]  (env passes through)

--legs: "gpu", "ref", or "gpu+VAR=v+VAR2=w" (a gpu leg with extra environment,
e.g. gpu+SMEM_GPU_DENSIFY=walk; gpu+B=<n> sets that leg's -b); the SAM of every
leg is compared with the first.
"""
import argparse
import hashlib
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument("--reads", type=int, default=200_000)
    p.add_argument("--threads", type=int, default=16)
    p.add_argument("--out", default=None)
    p.add_argument("--legs", default="gpu/ref")
    p.add_argument("--batch", type=int, default=0, help="bwa -b (default: reads / threads)")
    own, rest = p.parse_known_args()
    import torch
    torch.cuda.device_count()
    import bench
    from smemgpu import synth
    a = bench.parse(rest)
    a.reads = max(a.reads, own.reads)  # --reads past the bench's 1M: more chunks
    idx, _, sa, codes = bench.get_index(a, 0, lambda: None, 0)
    reads = bench.make_reads(a, 0, codes, 1)
    base = bench.genome_key(a)
    if not all(os.path.exists(base + e) for e in (".pac", ".ann", ".amb")):
        synth.write_bwa_bns(base + ".tmp", codes)
        for e in (".pac", ".ann", ".amb"):
            os.replace(base + ".tmp" + e, base + e)
    m = min(own.reads, reads.n)
    sub = reads.subset(range(m))
    bodies = {}
    with tempfile.TemporaryDirectory(dir=a.cache) as d:
        fq = os.path.join(d, "r.fq")
        synth.write_fastq(fq, sub)
        batch = own.batch or max(1024, -(-m // own.threads))
        print(f"[probe] {m} reads, -t {own.threads} -b {batch}", flush=True)
        legs = []
        for leg in own.legs.split("/"):
            name, *kv = leg.split("+")
            env = dict(os.environ, SMEM_GPU_TIMES="1", **dict(x.split("=", 1) for x in kv))
            b = env.pop("B", batch)  # gpu+B=<n>: this leg's bwa -b (B=auto: no -b)
            bopt = [] if str(b) == "auto" else ["-b", str(b)]
            cmd = ([bench.BWA_GPU, "mem", "-t", str(own.threads)] + bopt + [base, fq] if name == "gpu" else
                   [bench.REF_HARNESS, "mem", base, fq, str(own.threads), "1", "0"])
            legs.append((leg, cmd, env))
        for name, cmd, env in legs:
            t = time.time()
            p2 = subprocess.run(cmd, capture_output=True, env=env, timeout=900)
            body = b"\n".join(l for l in p2.stdout.split(b"\n") if not l.startswith(b"@PG"))
            err = p2.stderr.decode(errors="replace")
            keep = [l for l in err.split("\n") if "mem_batch_gpu" in l or "[W::" in l or "[E::" in l or "rror" in l
                    or "smem_gpu" in l or "mem_process_seqs" in l or "main_mem" in l or "real sec" in l
                    or "held" in l]
            nl = body.count(b"\n")
            print(f"== {name}: rc {p2.returncode}, {time.time() - t:.1f} s, sha {hashlib.sha256(body).hexdigest()[:16]}, "
                  f"{nl} lines", flush=True)
            for l in keep[:120]:
                print("   ", l, flush=True)
            bodies[name] = body
            if own.out:
                os.makedirs(own.out, exist_ok=True)
                with open(os.path.join(own.out, name + ".sam"), "wb") as fh:
                    fh.write(body)
                with open(os.path.join(own.out, name + ".err"), "w") as fh:
                    fh.write(err)
    first = legs[0][0]
    for name, _, _ in legs[1:]:
        print(f"== {first} vs {name}", flush=True)
        diff_summary(bodies[first], bodies[name], batch)


def diff_summary(gpu, ref, batch):
    """Which SAM records differ, and which worker batch (read index // -b) each belongs to."""
    if gpu == ref:
        print("== SAM identical", flush=True)
        return
    def records(body):
        rec = {}
        for l in body.split(b"\n"):
            if not l or l.startswith(b"@"):
                continue
            rec.setdefault(l.split(b"\t", 1)[0], []).append(l)
        return rec
    g, r = records(gpu), records(ref)
    names = list(dict.fromkeys(list(r) + list(g)))
    order = {n: i for i, n in enumerate(r)}
    bad = [n for n in names if g.get(n) != r.get(n)]
    print(f"== SAM differs: {len(bad)} of {len(names)} reads "
          f"(gpu {sum(map(len, g.values()))} records, ref {sum(map(len, r.values()))})", flush=True)
    by_batch = {}
    for n in bad:
        by_batch.setdefault(order.get(n, -1) // batch if n in order else -1, []).append(n)
    print("   differing reads by batch:", {k: len(v) for k, v in sorted(by_batch.items())}, flush=True)
    for n in bad[:6]:
        print(f"   read {n.decode(errors='replace')} (index {order.get(n)}):", flush=True)
        for l in r.get(n, []):
            print("     ref", l[:220].decode(errors="replace"), flush=True)
        for l in g.get(n, []):
            print("     gpu", l[:220].decode(errors="replace"), flush=True)


if __name__ == "__main__":
    main()

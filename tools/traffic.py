"""Record the seeding kernel's per-launch memory-side traffic for bench.py.

Runs two rocprofv3 counter passes (FETCH_SIZE, then WRITE_SIZE: they do not
fit one pass, MI355X_MICROARCH.md §counters) over tools/prof_run.py on the
bench workload and writes profiles/traffic.json, which bench.py reports as
roofline.traffic when its workload matches.

    python tools/traffic.py [--genome-mbp 1000 --reads 1000000] [--out profiles/traffic.json]

FETCH_SIZE is TCC_EA0_RDREQ x 64 B (KiB units): the L2's fabric-side read
requests, Infinity-Cache hits included.  The guide calibrates it at 1/2 of
the bytes for 16-B-per-lane coalesced streaming reads and leaves other access
shapes uncalibrated; the seeding kernel's are random 16-B lane chunks, so the
value is reported as measured.
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_pass(counter: str, out_dir: str, a) -> float:
    d = os.path.join(out_dir, counter)
    cmd = ["rocprofv3", "--pmc", counter, "--kernel-include-regex", "seed_kernel", "--output-format", "csv",
           "-d", d, "-o", "p", "--", sys.executable, os.path.join(ROOT, "tools", "prof_run.py"),
           "--genome-mbp", str(a.genome_mbp), "--reads", str(a.reads), "--read-len", str(a.read_len),
           "--seed", str(a.seed), "--launches", "1"]
    subprocess.run(cmd, check=True, timeout=600)
    tot, n = 0.0, set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                tot += float(r["Counter_Value"])
                n.add(r.get("Dispatch_Id", ""))
    # the main pass only (an overflow re-run would be a second dispatch)
    return tot * 1024.0, len(n)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--genome-mbp", type=float, default=3101.804739)
    p.add_argument("--reads", type=int, default=1_000_000)
    p.add_argument("--read-len", type=int, default=150)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--tmp", default=os.path.join(ROOT, "gpurun_out", "traffic"))
    p.add_argument("--out", default=os.path.join(ROOT, "profiles", "traffic.json"))
    a = p.parse_args()
    os.environ.setdefault("TMPDIR", "/tmp")
    fetch, nf = run_pass("FETCH_SIZE", a.tmp, a)
    write, nw = run_pass("WRITE_SIZE", a.tmp, a)
    out = {"bytes_per_launch": fetch, "write_bytes_per_launch": write, "dispatches": [nf, nw],
           "counter": "FETCH_SIZE x 1024 (TCC_EA0_RDREQ x 64 B), as measured",
           "workload": {"genome_mbp": a.genome_mbp, "reads": a.reads, "read_len": a.read_len, "seed": a.seed},
           "measured": time.strftime("%Y-%m-%d %H:%M:%S")}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

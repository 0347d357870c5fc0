"""Record the seeding kernel's per-launch memory-side counters for bench.py.

Runs rocprofv3 counter passes (one run per pass, nothing else combined with
--pmc: MI355X_MICROARCH.md §counters) over tools/prof_run.py on the bench
workload and writes profiles/traffic.json, which bench.py reports in
roofline.traffic / request_roofline when its workload AND its library build
(smem_gpu_build_id) match -- or its seeding kernel (smem_gpu_kernel_id: the
kernel's own sources and flags) and launch shape match, for runtime-only changes:

  pass 1: TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum  -- L2 fabric read requests
  pass 2: WRITE_SIZE
  pass 3: SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES

Calibration (profiles/r02/probe/fetch_size_calibration.txt): on random 16-B
and 32-B gathers of known count, TCC_EA0_RDREQ counts exactly one request per
gather and FETCH_SIZE = 64 B x TCC_EA0_RDREQ, i.e. each random request moves
one 64-B line; so traffic = 64 B x TCC_EA0_RDREQ.

    python tools/traffic.py [bench.py workload args] [--out profiles/traffic.json]
"""
import csv
import glob
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)


def run_pass(counters: list, out_dir: str, rest: list, extra: list = ()) -> dict:
    d = os.path.join(out_dir, "_".join(c.split("_")[0] + str(i) for i, c in enumerate(counters)))
    cmd = ["timeout", "-s", "KILL", "300", "rocprofv3", "--pmc", *counters, "--kernel-include-regex", "seed_(wp_)?kernel",
           "--output-format", "csv", "-d", d, "-o", "p", "--", sys.executable, os.path.join(ROOT, "tools", "prof_run.py"),
           "--launches", "1", *extra, *rest]
    subprocess.run(cmd, check=True)
    tot, disp = {}, {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Counter_Name"]
            tot[k] = tot.get(k, 0.0) + float(r["Counter_Value"])
            disp.setdefault(k, set()).add(r.get("Dispatch_Id", ""))
    return {k: (v, len(disp[k])) for k, v in tot.items()}


def main():
    import argparse
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument("--out", default=os.path.join(ROOT, "profiles", "traffic.json"))
    p.add_argument("--tmp", default=os.path.join(ROOT, "gpurun_out", "traffic"))
    own, rest = p.parse_known_args()
    import bench
    import smemgpu
    a = bench.parse(rest)
    os.environ.setdefault("TMPDIR", "/tmp")
    r1 = run_pass(["TCC_EA0_RDREQ_sum", "TCC_HIT_sum", "TCC_MISS_sum"], own.tmp, rest)
    launch_json = os.path.join(own.tmp, "launch.json")
    r2 = run_pass(["WRITE_SIZE"], own.tmp, rest, ["--stats-out", launch_json])
    sq_names = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES",
                "SQ_BUSY_CYCLES", "SQ_WAVES"]
    r3 = run_pass(sq_names, own.tmp, rest)
    with open(launch_json) as fh:
        launch = json.load(fh)
    out = {"rdreq_per_launch": r1["TCC_EA0_RDREQ_sum"][0], "tcc_hit_per_launch": r1["TCC_HIT_sum"][0],
           "tcc_miss_per_launch": r1["TCC_MISS_sum"][0], "write_bytes_per_launch": r2["WRITE_SIZE"][0] * 1024.0,
           "dispatches": [r1["TCC_EA0_RDREQ_sum"][1], r2["WRITE_SIZE"][1], r3["SQ_WAVES"][1]],
           "counter": "TCC_EA0_RDREQ_sum (L2 -> fabric read requests), TCC_HIT/MISS_sum, WRITE_SIZE x 1024; "
                      "sq: SQ_* per launch (instructions; *_CYCLES / WAIT / ACTIVE in quad-cycles)",
           "sq": {k: r3[k][0] for k in sq_names if k in r3},
           "workload": {"genome_mbp": a.genome_mbp, "reads": a.reads, "read_len": a.read_len, "seed": a.seed,
                        "sub": a.sub, "genome_profile": a.genome_profile},
           "build_id": launch["build_id"],  # the library the counted launches ran on
           "kernel_id": launch["kernel_id"],
           "variant": launch.get("variant"),  # the seeding kernel the counted launches ran
           "launch": {"grid": launch["grid"], "block": launch["block"]},
           "measured": time.strftime("%Y-%m-%d %H:%M:%S")}
    os.makedirs(os.path.dirname(own.out) or ".", exist_ok=True)
    with open(own.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

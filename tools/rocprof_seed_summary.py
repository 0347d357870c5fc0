"""Summarise a rocprofv3 kernel trace of bench.py's timed seeding steps beside
the bench line of the same command: the seeding kernel's launches split into
warm-up (alone), the second worker's start and the timed ones, their mean
duration against the line's HIP-event kernel_ms, and the union of the timed
launches against kernel_busy_ms (profiles/<round>/rocprof/*_summary.txt).

    python tools/rocprof_seed_summary.py <prof_dir> <bench_line.json> [--warmup W] [--steps K] > summary.txt
"""
import argparse
import csv
import glob
import json
import os


def main():
    p = argparse.ArgumentParser()
    p.add_argument("prof_dir")
    p.add_argument("line")
    p.add_argument("--warmup", type=int, default=None)
    p.add_argument("--steps", type=int, default=None)
    a = p.parse_args()
    d = json.loads(open(a.line).read().strip().splitlines()[-1])
    W = a.warmup if a.warmup is not None else d["warmup"]
    K = a.steps if a.steps is not None else d["steps"]
    tr = glob.glob(os.path.join(a.prof_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(tr)) if "seed_wp_kernel" in r["Kernel_Name"] or "seed_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    dur = [(e - s) / 1e6 for s, e in iv]
    per_step = max(1, (len(rows) - W - 1) // K) if len(rows) > W + 1 else 1
    timed = iv[len(iv) - K * per_step:]
    merged = []
    for s, e in sorted(timed):
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    union = sum(e - s for s, e in merged) / 1e6
    r = d["roofline"]
    print(f"kernel trace: {os.path.relpath(tr)}")
    print(f"build_id {d.get('build_id')}  kernel_id {d.get('kernel_id')}  workload: {d['config']['workload']}")
    print(f"seed launches: {len(rows)} (warm-up {W} alone, then {per_step} per timed step x {K}); every launch = "
          f"{d['config'].get('reads_per_gpu', 0) // per_step if per_step else 0} reads")
    print(f"  warm-up (alone) durations ms: {[round(x, 3) for x in dur[:W]]}   bench kernel_ms_alone {r.get('kernel_ms_alone')}")
    td = [(e - s) / 1e6 for s, e in timed]
    print(f"  timed launches mean duration {sum(td) / len(td):.3f} ms   bench kernel_ms (HIP events, same launches) "
          f"{r.get('kernel_ms')}")
    print(f"  timed launches union / {K} = {union / K * (1 if per_step == 1 else 1):.3f} ms   bench kernel_busy_ms "
          f"(chip clock spans) {r.get('kernel_busy_ms')}")
    print(f"  all {len(rows)} launches mean {sum(dur) / len(dur):.3f} ms (= kernel_stats.csv AverageNs)")
    print(f"line: value {d['value']} {d['unit']}, ms_per_step {d['ms_per_step']}, roofline frac {r.get('frac')}, "
          f"request frac {r.get('request_roofline', {}).get('frac')}")


if __name__ == "__main__":
    main()

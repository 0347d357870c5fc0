"""Summarise seed_kernel from a rocprofv3 --kernel-trace run of bench.py beside
the bench line that run printed: warmup launches (alone), the timed
launches' mean duration (what the bench's HIP events give) and their union
on the trace clock divided by the launch count (what the bench's chip-clock
busy time gives).

    python tools/rocprof_summary.py <prof>/c2_kernel_trace.csv <prof_bench.json> [--warmup 2] [--cmd "..."]
"""
import argparse
import csv
import json


def union_ns(spans):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(spans):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    return tot + (cur_e - cur_s if cur_e is not None else 0)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("bench_json")
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--kernel", default="seed_", help="kernel-name substring (seed_kernel / seed_wp_kernel)")
    p.add_argument("--cmd", default="")
    a = p.parse_args()
    spans = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            if a.kernel in r["Kernel_Name"] and ("seed_kernel" in r["Kernel_Name"] or "seed_wp_kernel" in r["Kernel_Name"]
                                                 or a.kernel != "seed_"):
                spans.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    spans.sort()
    b = json.load(open(a.bench_json))
    r = b["roofline"]
    steps = b["steps"]
    timed = spans[-steps:]
    warm = spans[:a.warmup]
    dur = lambda s: (s[1] - s[0]) / 1e6
    out = []
    if a.cmd:
        out.append(a.cmd)
    out.append(f"build_id {b['build_id']}  workload: {b['config']['workload']}")
    out.append(f"{a.kernel} launches: {len(spans)} ({a.warmup} warmup alone, "
               f"{len(spans) - a.warmup - steps} second-worker start, {steps} timed); every launch = "
               f"{b['config']['reads_per_gpu'] // 1000000}M reads")
    out.append(f"  warmup (alone) durations ms: {[round(dur(s), 3) for s in warm]}  "
               f"bench kernel_ms_alone {r['kernel_ms_alone']:.3f}")
    out.append(f"  timed launches mean duration {sum(map(dur, timed)) / len(timed):.3f} ms   "
               f"bench kernel_ms (HIP events, same launches) {r['kernel_ms']:.3f}")
    out.append(f"  timed launches union / {steps} = {union_ns(timed) / 1e6 / steps:.3f} ms   "
               f"bench kernel_busy_ms (chip clock spans) {r['kernel_busy_ms']:.3f}")
    out.append(f"  all {len(spans)} launches mean {sum(map(dur, spans)) / len(spans):.3f} ms "
               f"(= kernel_stats.csv AverageNs)")
    print("\n".join(out))


if __name__ == "__main__":
    main()

"""Timeline of one streaming pass from a rocprofv3 --kernel-trace CSV:
per seed_kernel launch its start / duration / concurrency, the union of
seeding time over the pass, and the time the other kernels (blit copies,
compaction, finalize) took inside it.

    python tools/trace_stream.py <dir with *_kernel_trace.csv> [--last N]
"""
import argparse
import csv
import glob
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    tot, (cs, ce) = 0, iv[0]
    for a, b in iv[1:]:
        if a > ce:
            tot += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    return tot + ce - cs


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--last", type=int, default=0, help="seed_kernel launches of the pass (default: since the last gap > 50 ms)")
    a = p.parse_args()
    K = []
    for f in glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True):
        K += list(csv.DictReader(open(f)))
    for k in K:
        k["a"], k["b"] = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
    K.sort(key=lambda k: k["a"])
    seed = [k for k in K if "seed_kernel" in k["Kernel_Name"] or "seed_wp_kernel" in k["Kernel_Name"]]
    if a.last:
        s = seed[-a.last:]
    else:  # the last run of launches without a 50 ms gap
        i = len(seed) - 1
        while i > 0 and seed[i]["a"] - seed[i - 1]["b"] < 50e6:
            i -= 1
        s = seed[i:]
    t0, t1 = s[0]["a"], max(k["b"] for k in s)
    print(f"{len(s)} seed launches, span {(t1 - t0) / 1e6:.1f} ms, seeding union {union([(k['a'], k['b']) for k in s]) / 1e6:.1f} ms, "
          f"sum {sum(k['b'] - k['a'] for k in s) / 1e6:.1f} ms")
    for k in s:
        conc = sum(1 for o in s if o is not k and o["a"] < k["b"] and o["b"] > k["a"])
        print(f"  stream {k['Stream_Id']:>3} grid {int(k['Grid_Size_X']) // 256:>5} start {(k['a'] - t0) / 1e6:8.2f} "
              f"dur {(k['b'] - k['a']) / 1e6:7.2f} overlaps {conc}")
    agg = defaultdict(lambda: [0, 0.0, []])
    for k in K:
        if k["a"] >= t0 and k["a"] <= t1:
            n = k["Kernel_Name"][:70]
            agg[n][0] += 1
            agg[n][1] += (k["b"] - k["a"]) / 1e6
            agg[n][2].append((k["a"], k["b"]))
    for n, (c, d, iv) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"  {c:5d} x  {d:8.2f} ms (union {union(iv) / 1e6:7.2f})  {n}")


if __name__ == "__main__":
    main()

"""Sum rocprofv3 counter CSVs per counter (all dispatches of the filtered kernel;
--by-kernel: per kernel name).
    python tools/pmc_sum.py [--by-kernel] gpurun_out/pmc_dir [...]"""
import collections
import csv
import glob
import json
import sys

by_kernel = "--by-kernel" in sys.argv
for d in [a for a in sys.argv[1:] if a != "--by-kernel"]:
    agg = collections.defaultdict(float)
    n = collections.defaultdict(set)
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = (r.get("Kernel_Name", "") + " | " if by_kernel else "") + r["Counter_Name"]
            agg[k] += float(r["Counter_Value"])
            n[k].add((f, r.get("Dispatch_Id", "")))
    print(d, json.dumps({k: [v, len(n[k])] for k, v in sorted(agg.items())}, indent=1))

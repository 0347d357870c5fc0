"""Sum rocprofv3 counter CSVs per counter (all dispatches of the filtered kernel).
    python tools/pmc_sum.py gpurun_out/pmc_dir [...]"""
import collections
import csv
import glob
import json
import sys

for d in sys.argv[1:]:
    agg = collections.defaultdict(float)
    n = collections.defaultdict(set)
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]].add((f, r.get("Dispatch_Id", "")))
    print(d, json.dumps({k: [v, len(n[k])] for k, v in sorted(agg.items())}, indent=1))

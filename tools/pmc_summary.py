#!/usr/bin/env python3
"""Summarise rocprofv3 counter CSVs (gpurun_out/pmc*/run_counter_collection.csv)
for one kernel: per-dispatch averages of every counter collected."""
import collections
import csv
import glob
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else "k_stream"
root = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
vals = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/pmc*/run_counter_collection.csv")):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        vals[c].append(v)
for c in sorted(vals):
    v = vals[c]
    print(f"{c:28s} {sum(v) / len(v):14.4g}   (dispatches={len(v)})")

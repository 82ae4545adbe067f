#!/usr/bin/env python3
"""Summarise a tools/sq_pass.sh run: per-dispatch means of the 8 SQ counters
over a kernel's full-size launches (the largest grid of the run), and the
wave-time split DESIGN.md quotes (shares of SQ_WAVE_CYCLES: parked on
s_waitcnt / barrier, ready but not issued, issuing).

    python tools/sq_summary.py gpurun_out/sq8 ["k_stream<false, true, 3, 0>"]
"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
kernel = sys.argv[2] if len(sys.argv) > 2 else "k_stream<false, true, 0, 0>"
vals = collections.defaultdict(lambda: collections.defaultdict(float))
grid = {}
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if kernel in r["Kernel_Name"]:
            vals[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            grid[r["Dispatch_Id"]] = int(r["Grid_Size"])
if not grid:
    sys.exit(f"no dispatch of {kernel} under {root}")
big = max(grid.values())
ds = [d for d in vals if grid[d] == big]
mean = {c: sum(vals[d][c] for d in ds) / len(ds) for c in vals[ds[0]]}
print(f"{kernel}: {len(ds)} full-size dispatches (grid {big}), per-dispatch means")
for c in sorted(mean):
    print(f"  {c:22s} {mean[c]:.4g}")
w = mean.get("SQ_WAVE_CYCLES")
if w:
    print("shares of SQ_WAVE_CYCLES:")
    for c, name in (("SQ_WAIT_ANY", "parked on s_waitcnt / barrier"), ("SQ_WAIT_INST_ANY", "ready, not issued"),
                    ("SQ_ACTIVE_INST_ANY", "issuing"), ("SQ_ACTIVE_INST_VALU", "  of which VALU"),
                    ("SQ_ACTIVE_INST_LDS", "  of which LDS")):
        if c in mean:
            print(f"  {name:32s} {mean[c] / w:.3f}")

#!/usr/bin/env python3
"""Per-kernel durations from a rocprofv3 kernel trace (run_kernel_trace.csv).

The --stats average of k_stream covers every dispatch of the profiled bench
run: the validation launches right after a cold start and the warm-up, while
the clocks still ramp (DESIGN.md §7 "clock ramp"), as well as the timed ones.
bench.py's roofline.kernel_ms is the HIP-event average of the LAST `tail`
dispatches of the kernel (its split timing), so this prints, per kernel, the
mean over all dispatches and over the last `tail`, which is the number to
compare with kernel_ms.

  usage: prof_summary.py run_kernel_trace.csv [tail=10] > summary.json
"""
import collections
import csv
import json
import sys


def main(argv):
    path = argv[1]
    tail = int(argv[2]) if len(argv) > 2 else 10
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        dur[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    out = {}
    for name, v in sorted(dur.items(), key=lambda kv: -sum(d for _, d in kv[1])):
        v.sort()
        d = [x for _, x in v]
        out[name[:120]] = {"calls": len(d), "mean_us_all": sum(d) / len(d) / 1e3,
                           f"mean_us_last_{min(tail, len(d))}": sum(d[-tail:]) / len(d[-tail:]) / 1e3,
                           "min_us": min(d) / 1e3}
    json.dump(out, sys.stdout, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))

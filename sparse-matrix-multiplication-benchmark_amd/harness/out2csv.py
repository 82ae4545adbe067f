#!/usr/bin/env python3
"""out.txt -> CSV for the benchmark harness.

The reference's parse-out2csv.sh (parse-out2csv.sh:3-20) joins every five
lines of SparseGEMM.cpp's output; main.cpp prints a different layout (a test
header, a "Matrix info" line, a table, then six legacy lines,
main.cpp:190-196,296,409-432), so that script produces garbage on the
harness's own out.txt.  This parser keys on content instead of line counts
and reads either program's output (main.cpp linked against libtcsc_amd.so,
or harness/tcsc_bench):

  [TEST i/n] Matrix Size: MxKxN ...          -> M, K, N of the case
  [*] Matrix info: NNZ non-zeros out of ...  -> nonZero
  NAME cycles=C, flops=F, performance=P      -> one column group per NAME

One CSV row per case: M,K,N,nonZero, then cycles_/flops_/performance_ for
each algorithm in the order first seen.  Lines that match nothing are
ignored (banners, progress bars, tables); a legacy line before any test
header is an error.

  usage: out2csv.py [out.txt] > results.csv      (stdin when no file)
"""
from __future__ import annotations

import re
import sys

RE_CASE = re.compile(r"Matrix Size:\s*(\d+)x(\d+)x(\d+)")
RE_NNZ = re.compile(r"Matrix info:\s*(\d+)\s+non-zeros")
RE_LEGACY = re.compile(r"^\s*([A-Za-z][\w]*)\s+cycles=([-+\d.eE]+),\s*flops=(-?\d+),\s*performance=([-+\d.eEnaif]+)\s*$")


def parse(lines):
    """Returns (algorithms in first-seen order, list of case dicts)."""
    cases, algos = [], []
    cur = None
    for line in lines:
        m = RE_CASE.search(line)
        if m:
            cur = {"M": int(m.group(1)), "K": int(m.group(2)), "N": int(m.group(3)), "nonZero": "", "algo": {}}
            cases.append(cur)
            continue
        m = RE_NNZ.search(line)
        if m and cur is not None:
            cur["nonZero"] = int(m.group(1))
            continue
        m = RE_LEGACY.match(line)
        if m:
            if cur is None:
                raise ValueError(f"legacy line before any test header: {line.strip()!r}")
            name = m.group(1)
            if name not in algos:
                algos.append(name)
            cur["algo"][name] = (m.group(2), m.group(3), m.group(4))
    return algos, cases


def to_csv(algos, cases) -> str:
    head = ["M", "K", "N", "nonZero"]
    for a in algos:
        head += [f"cycles_{a}", f"flops_{a}", f"performance_{a}"]
    out = [",".join(head)]
    for c in cases:
        row = [str(c["M"]), str(c["K"]), str(c["N"]), str(c["nonZero"])]
        for a in algos:
            row += list(c["algo"].get(a, ("", "", "")))
        out.append(",".join(row))
    return "\n".join(out) + "\n"


def main(argv) -> int:
    if len(argv) > 2:
        print(__doc__, file=sys.stderr)
        return 2
    f = open(argv[1], encoding="utf-8", errors="replace") if len(argv) == 2 else sys.stdin
    try:
        algos, cases = parse(f)
    finally:
        if f is not sys.stdin:
            f.close()
    sys.stdout.write(to_csv(algos, cases))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))

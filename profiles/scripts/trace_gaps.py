#!/usr/bin/env python3
"""trace_gaps.py <run_kernel_trace.csv> [last N] — the last N kernel dispatches of a
rocprofv3 --kernel-trace run in time order: duration of each and the idle gap before it
(the GPU timeline of back-to-back calls: launch boundaries, empty tail kernels)."""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    m = re.match(r"(?:void )?(?:fmx::)?([\w:]+)(<[^(]*>)?", name)
    base = m.group(1) if m else name[:40]
    targs = (m.group(2) or "") if m else ""
    return (base + targs)[:70]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-n:]
    prev_end = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        print("%8.2f us  gap %7.2f us  %s grid=%s" % ((e - s) / 1e3, gap, short(r["Kernel_Name"]), r["Grid_Size_X"]))
        prev_end = e


if __name__ == "__main__":
    main()

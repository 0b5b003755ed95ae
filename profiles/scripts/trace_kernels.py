#!/usr/bin/env python3
"""trace_kernels.py <rocprofv3 -d dir>: per query kernel (template arguments kept) the
dispatch count and the median / min duration from the kernel trace."""
import csv
import glob
import re
import statistics
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
by = {}
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    m = re.search(r"(k_\w+)<([^>]*)>", n) or re.search(r"(k_\w+)\(", n)
    if not m or not any(k in n for k in ("k_count", "k_locate", "k_walk", "k_scan", "k_extract")):
        continue
    key = m.group(1) + ("<" + m.group(2).replace("fmx::(anonymous namespace)::", "") + ">" if m.lastindex > 1 else "")
    by.setdefault(key, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(by.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1])):
    print("%5d  median %9.1f us  min %9.1f us  %s" % (len(v), statistics.median(v) / 1e3, min(v) / 1e3, k))

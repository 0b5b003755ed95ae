"""Median per-dispatch sums of the SQ counters in a rocprofv3 --pmc csv, per kernel.
Usage: pmc_sq.py run_counter_collection.csv"""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    agg[(r["Kernel_Name"][:70], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
per = collections.defaultdict(lambda: collections.defaultdict(list))
for (k, _), cs in agg.items():
    for c, v in cs.items():
        per[k][c].append(v)
for k, cs in per.items():
    n = len(next(iter(cs.values())))
    med = {c: statistics.median(v) for c, v in cs.items()}
    w = med.get("SQ_WAVES", 0) or 1
    print(k, "dispatches=%d" % n)
    print("   " + "  ".join("%s=%.3g" % (c, v) for c, v in sorted(med.items())))
    print("   per wave: " + "  ".join("%s=%.0f" % (c, v / w) for c, v in sorted(med.items()) if c.startswith("SQ_INSTS")))

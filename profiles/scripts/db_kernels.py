"""Per-kernel dispatch durations from a rocprofv3 rocpd database (run_results.db):
median / mean / count per kernel name matching a regex.  Usage: db_kernels.py DB [REGEX]"""
import glob
import re
import sqlite3
import statistics
import sys

db = sys.argv[1]
if not db.endswith(".db"):
    db = glob.glob(db + "/**/*.db", recursive=True)[0]
rx = re.compile(sys.argv[2] if len(sys.argv) > 2 else "k_")
c = sqlite3.connect(db)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
rows = c.execute(f"select s.kernel_name, d.end - d.start from {kd} d join {ks} s on d.kernel_id = s.id").fetchall()
by = {}
for name, dur in rows:
    if rx.search(name):
        by.setdefault(name, []).append(dur)
for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    print("%8.1f us median  %8.1f mean  n=%4d  %s" % (statistics.median(v) / 1e3, statistics.mean(v) / 1e3, len(v), name[:150]))

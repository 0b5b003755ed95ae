#!/bin/bash
# calib_fetch.sh — FETCH_SIZE calibration for random W-byte reads (W = 16..128):
# runs profiles/microbench/gather_bench under rocprofv3 --pmc FETCH_SIZE (own pass)
# and prints FETCH_SIZE*1024 / (reads*W) per dispatch of k_indep.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/calib_fetch
mkdir -p "$OUT"
hipcc -O3 --offload-arch=gfx950 "$ROOT/profiles/microbench/gather_bench.hip" -o "$OUT/gather_bench"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_indep --output-format csv -d "$OUT/pmc" -o run -- "$OUT/gather_bench" 4 256 > "$OUT/gather.txt" 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-include-regex k_indep --output-format csv -d "$OUT/pmc2" -o run -- "$OUT/gather_bench" 4 256 > "$OUT/gather2.txt" 2>&1 || true
python3 - "$OUT" <<'PY'
import csv, glob, sys, re
out = sys.argv[1]
for sub in ("pmc", "pmc2"):
    rows = []
    for f in glob.glob(out + "/" + sub + "/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    for r in rows:
        name = r["Kernel_Name"]
        m = re.search(r"k_indep<(\d+)>", name)
        W = int(m.group(1)) if m else 0
        print(sub, r.get("Dispatch_Id"), "W=%d" % W, r["Counter_Name"], r["Counter_Value"])
PY

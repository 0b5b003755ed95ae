#!/bin/bash
# ceiling_ab.sh <tag> [rounds] — the headline count against the ceiling of its own access mix,
# in one box session: per round, profiles/microbench/mix_bench (the same 12.5 M x (8-B offset +
# 20-B pattern + one random 16-B record out of 17.2 GB + 8-B count) in the production shape and
# the two halves alone) and `bench.py --only count` (HIP-event median of 30 launches), each in
# a fresh process.  Output: gpurun_out/ceiling_<tag>.jsonl
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/ceiling_$1.jsonl
: > "$OUT"
for r in $(seq 1 ${2:-2}); do
  timeout -k 10 200 "$ROOT/profiles/microbench/mix_bench" 12.5 21 | sed "s/^{/{\"round\": $r, \"src\": \"mix_bench\", /" >> "$OUT" || exit 1
  R=$(timeout -k 10 240 python3 "$ROOT/bench.py" --only count --steps 30 --warmup 5 2>/dev/null | tail -1) || exit 1
  python3 -c "
import json,sys; d=json.loads(sys.argv[1])['count']
print(json.dumps({'round': $r, 'src': 'bench_count', 'kernel_ms_median': d['kernel_ms_median'], 'kernel_ms_min': d['kernel_ms_min']}))" "$R" >> "$OUT"
done

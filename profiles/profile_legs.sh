#!/bin/bash
# profile_legs.sh <tag> <leg,leg,...> [bench.py args...]
#
# Per-leg kernel profiles of bench.py on the GPU box (MI355X_MICROARCH.md §rocprofv3):
# for every leg, `bench.py --only <leg>` runs under three passes of its own —
#   1  rocprofv3 --kernel-trace --stats          per-kernel durations
#   2  rocprofv3 --pmc FETCH_SIZE                 HBM read bytes (own pass)
#   3  rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum   L2 hit rate (own pass)
# then profiles/summarize_legs.py writes gpurun_out/prof_legs_<tag>/pmc_legs.json (the
# traffic bench.py reports per leg, keyed "<workload>|<leg>") and stats.json.  Counter
# passes never combine --pmc with sys/runtime/hip traces.  Leg "count" = the headline.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1
LEGS=$2
shift 2
OUT=$ROOT/gpurun_out/prof_legs_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
KRE="k_count|k_walk|k_locate|k_expand|k_scan"
for LEG in ${LEGS//,/ }; do
  D=$OUT/$LEG
  mkdir -p "$D"
  BENCH=(python3 "$ROOT/bench.py" --only "$LEG" --steps ${PROF_STEPS:-6} --warmup ${PROF_WARMUP:-1} "$@")
  echo "[profile_legs] $LEG" >&2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/trace" -o run -- "${BENCH[@]}" > "$D/bench_trace.json" 2> "$D/trace.err"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" --output-format csv -d "$D/pmc_fetch" -o run -- "${BENCH[@]}" > "$D/bench_fetch.json" 2> "$D/fetch.err"
  timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$KRE" --output-format csv -d "$D/pmc_l2" -o run -- "${BENCH[@]}" > "$D/bench_l2.json" 2> "$D/l2.err"
done
python3 "$ROOT/profiles/summarize_legs.py" "$OUT" "$TAG"

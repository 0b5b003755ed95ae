#!/bin/bash
# profile_count.sh <tag> [bench.py args...]
#
# Profiles the count kernel of bench.py on the GPU box (MI355X_MICROARCH.md
# §rocprofv3 / cdna_hip_programming.md §7):
#   pass 1  rocprofv3 --kernel-trace --stats           per-kernel durations
#   pass 2  rocprofv3 --pmc FETCH_SIZE                  HBM read bytes (own pass)
#   pass 3  rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum    L2 hit rate (own pass)
# then profiles/summarize.py writes gpurun_out/prof_<tag>/summary.json and the
# stats CSV; copy them into profiles/ to commit.  Counter passes never combine
# --pmc with sys/runtime/hip traces.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1
shift
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH=(python3 "$ROOT/bench.py" --no-cpu --p50-calls 0 "$@")
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "${BENCH[@]}" > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_count|k_walk_lines|k_walk<|k_locate|k_build_lctx|k_extract" --output-format csv -d "$OUT/pmc_fetch" -o run -- "${BENCH[@]}" > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 900 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_count|k_walk_lines|k_walk<|k_locate|k_build_lctx|k_extract" --output-format csv -d "$OUT/pmc_l2" -o run -- "${BENCH[@]}" > "$OUT/bench_l2.json" 2> "$OUT/l2.err"
python3 "$ROOT/profiles/summarize.py" "$OUT" "$TAG"

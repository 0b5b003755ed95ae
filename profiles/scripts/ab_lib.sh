#!/bin/bash
# ab_lib.sh <tag> <variant> [<variant> ...] — A/B of library builds on the GPU box: for each
# round, each variant's libcs_fmindex_<variant>.so is copied over the package's library in
# the box's copy of the tree and `bench.py --only <AB_LEG, default count>` runs in a fresh
# process (kernel time from HIP events).  Output: gpurun_out/ab_lib_<tag>.jsonl (one line
# per run).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
PKG=$ROOT/compressed-fm-index-implementation-with-learned-optimizations_amd
TAG=$1
shift
OUT=$ROOT/gpurun_out/ab_lib_$TAG.jsonl
: > "$OUT"
cp "$PKG/libcs_fmindex.so" "$PKG/libcs_fmindex_ab_saved.so"  # (restored at the end)
for round in $(seq 1 ${AB_ROUNDS:-2}); do
  for V in "$@"; do
    cp "$PKG/libcs_fmindex_$V.so" "$PKG/libcs_fmindex.so"
    echo "[ab_lib] round $round $V" >&2
    R=$(timeout -k 10 240 python3 "$ROOT/bench.py" --only "${AB_LEG:-count}" --steps 30 --warmup 5 ${AB_ARGS:-} | tail -1)
    echo "{\"variant\": \"$V\", \"round\": $round, \"result\": $R}" >> "$OUT"
  done
done
cp "$PKG/libcs_fmindex_ab_saved.so" "$PKG/libcs_fmindex.so"

#!/bin/bash
# pmc_probe.sh <tag> <leg,leg,...> <pass> [<pass> ...] — counter passes over single bench.py
# legs on the GPU box (one rocprofv3 --pmc run per pass, kernel-trace free, per the
# MI355X guide's slot limits: <= 8 SQ, 4 TCP, 2 TA counters per pass).  A pass is a
# comma-separated counter list.  Output: gpurun_out/pmc_probe_<tag>/<leg>/<n>/...csv
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1
LEGS=$2
shift 2
OUT=$ROOT/gpurun_out/pmc_probe_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for LEG in ${LEGS//,/ }; do
  n=0
  for PASS in "$@"; do
    n=$((n + 1))
    D=$OUT/$LEG/$n
    mkdir -p "$D"
    echo "[pmc_probe] $LEG pass $n: $PASS" >&2
    timeout -s KILL 240 rocprofv3 --pmc ${PASS//,/ } --kernel-include-regex "k_count" --output-format csv \
      -d "$D" -o run -- python3 "$ROOT/bench.py" --only "$LEG" --steps 4 --warmup 1 > "$D/bench.json" 2> "$D/err.txt"
  done
done

#!/bin/bash
# trace_leg.sh <tag> <leg> [env=val ...]: rocprofv3 kernel trace of one bench.py leg (--only),
# per-kernel medians printed (profiles/scripts/trace_kernels.py)
set -uo pipefail
TAG=$1; LEG=$2; shift 2
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
env "$@" true
for kv in "$@"; do export "$kv"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$LEG -o run -- \
  python3 $R/bench.py --only $LEG --steps 20 --warmup 3 ${TRACE_ARGS:-} > $O/$LEG.json 2> $O/$LEG.err || exit 1
python3 $R/profiles/scripts/trace_kernels.py $O/trace_$LEG

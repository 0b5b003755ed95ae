#!/bin/bash
# r05z: walk-line one-call locate, the emit's multi-position walks in per-tile slots for
# k_locate_walks — parity (walk-line variants, C5 full size), the C5 kernel trace and the C5
# library A/B (chain = round-5 before, walks = now)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r05z
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "one_call or context_windows or every_text" > $O/parity.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 250 --timeout-method thread \
  -k "c5" > $O/scale.log 2>&1 &&
TRACE_ARGS="--text-bytes 31999999999" timeout -k 10 400 bash profiles/scripts/trace_leg.sh r05z_walks locate_one \
  > $O/trace_walks.txt 2>&1 &&
AB_LEG=locate_one AB_ROUNDS=2 AB_ARGS="--text-bytes 31999999999" timeout -k 10 800 \
  bash profiles/scripts/ab_lib.sh r05z_c5_locate_one chain walks 2> $O/ab.err

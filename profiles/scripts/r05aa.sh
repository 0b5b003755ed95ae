#!/bin/bash
# r05aa: barrier-free one-call search over walk lines with the LF step's constants in
# registers (WalkK) — walk-line parity, then the C5 trace and library A/B (walks = the
# previous commit, walkk = now)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r05aa
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "one_call or context_windows or every_text" > $O/parity.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 250 --timeout-method thread \
  -k "c5" > $O/scale.log 2>&1 &&
TRACE_ARGS="--text-bytes 31999999999" timeout -k 10 400 bash profiles/scripts/trace_leg.sh r05aa_walkk locate_one \
  > $O/trace_walkk.txt 2>&1 &&
AB_LEG=locate_one AB_ROUNDS=2 AB_ARGS="--text-bytes 31999999999" timeout -k 10 800 \
  bash profiles/scripts/ab_lib.sh r05aa_c5_locate_one walks walkk 2> $O/ab.err

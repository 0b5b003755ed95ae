#!/bin/bash
# r05ae: the emit kernel loads its tile's base with the records (not after the block scan) —
# one-call locate parity, then the library A/B (head = the round's last commit, hoist = now)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r05ae
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "one_call or locate_records or context_windows" > $O/parity.log 2>&1 &&
AB_LEG=locate_one AB_ROUNDS=3 timeout -k 10 700 bash profiles/scripts/ab_lib.sh r05ae_locate_one head hoist 2> $O/ab.err

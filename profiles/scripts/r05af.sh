#!/bin/bash
# r05af: the routed count's listed counters spread over 256 lines (16 before: a batch whose
# every wave lists — long patterns, repetitive DNA — put ~6 k atomics on each) — routed
# parity, then library A/Bs (head = the round's last commit, l256 = now): 150-mers,
# repetitive DNA, the headline
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r05af
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "repetitive or majority or rout or verify_long or one_call" \
  > $O/parity.log 2>&1 &&
AB_LEG=count_m150 AB_ROUNDS=2 timeout -k 10 500 bash profiles/scripts/ab_lib.sh r05af_m150 head l256 2> $O/ab1.err &&
AB_LEG=count_rdna AB_ROUNDS=2 timeout -k 10 500 bash profiles/scripts/ab_lib.sh r05af_rdna head l256 2> $O/ab2.err &&
AB_LEG=count AB_ROUNDS=2 timeout -k 10 400 bash profiles/scripts/ab_lib.sh r05af_count head l256 2> $O/ab3.err

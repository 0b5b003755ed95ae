#!/bin/bash
# r05ab: the staged kernels issue their offsets loads before the block's map / barrier
# prologue — routed-count parity, then library A/Bs (head = the round's last commit, pre =
# with the early loads) on the headline and repetitive DNA
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r05ab
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "every_text or repetitive or majority or rout or packed or fixed" \
  > $O/parity.log 2>&1 &&
AB_LEG=count AB_ROUNDS=3 timeout -k 10 600 bash profiles/scripts/ab_lib.sh r05ab_count head pre 2> $O/ab1.err &&
AB_LEG=count_rdna AB_ROUNDS=2 timeout -k 10 500 bash profiles/scripts/ab_lib.sh r05ab_rdna head pre 2> $O/ab2.err

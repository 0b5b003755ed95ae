#!/bin/bash
# r05ad: three listed general searches per lane in the list kernel — routed-count parity,
# then library A/Bs (head = the round's last commit, g3 = three per lane) on repetitive DNA
# and the headline
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r05ad
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "every_text or repetitive or majority or rout or verify_long" \
  > $O/parity.log 2>&1 &&
AB_LEG=count_rdna AB_ROUNDS=2 timeout -k 10 500 bash profiles/scripts/ab_lib.sh r05ad_rdna head g3 2> $O/ab1.err &&
AB_LEG=count AB_ROUNDS=2 timeout -k 10 400 bash profiles/scripts/ab_lib.sh r05ad_count head g3 2> $O/ab2.err

#!/bin/bash
# r05ac: the barrier-free count forms build a per-wave symbol map after their offsets (no
# block barrier; a wave of long patterns reads no map) — parity of the count forms, then
# library A/Bs (head = the round's last commit, wmap = the per-wave map): headline, 150-mers,
# repetitive DNA
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r05ac
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "every_text or repetitive or majority or rout or packed or fixed or random_large or verify_long" \
  > $O/parity.log 2>&1 &&
AB_LEG=count AB_ROUNDS=3 timeout -k 10 600 bash profiles/scripts/ab_lib.sh r05ac_count head wmap 2> $O/ab1.err &&
AB_LEG=count_m150 AB_ROUNDS=2 timeout -k 10 500 bash profiles/scripts/ab_lib.sh r05ac_m150 head wmap 2> $O/ab2.err

#!/bin/bash
# r05ag: the routed long-pattern list kernel (k_count_long kList) held to 5 waves per SIMD and
# launched 5 blocks per CU (w5) against 4 and 4 (head): its 128 VGPRs (SGPR spills of the list
# loop) against the direct form's 92 at 5 waves — 150-mers routed 1.66 ms in the kernel against
# 1.55 direct.  Routed parity with w5, then library A/Bs: 150-mers, repetitive DNA (its general
# searches run in the same kernel), the headline
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
PKG=$R/compressed-fm-index-implementation-with-learned-optimizations_amd
O=$R/gpurun_out/r05ag
mkdir -p $O
cd $R
cp $PKG/libcs_fmindex.so $PKG/libcs_fmindex_saved0.so
cp $PKG/libcs_fmindex_w5.so $PKG/libcs_fmindex.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "repetitive or majority or rout or verify_long or selectors" \
  > $O/parity_w5.log 2>&1 &&
cp $PKG/libcs_fmindex_saved0.so $PKG/libcs_fmindex.so &&
AB_LEG=count_m150 AB_ROUNDS=2 timeout -k 10 500 bash profiles/scripts/ab_lib.sh r05ag_m150 head w5 2> $O/ab1.err &&
AB_LEG=count_rdna AB_ROUNDS=2 timeout -k 10 500 bash profiles/scripts/ab_lib.sh r05ag_rdna head w5 2> $O/ab2.err &&
AB_LEG=count AB_ROUNDS=2 timeout -k 10 400 bash profiles/scripts/ab_lib.sh r05ag_count head w5 2> $O/ab3.err

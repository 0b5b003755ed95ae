#!/bin/bash
# r05t: the list kernel's chain payload (no offsets / pattern bytes read before a listed
# general search's steps) and the barrier-free one-call search over walk lines — parity of
# the routed count and one-call locate paths, then library A/Bs (base = the previous commit,
# chain = + the chain payload, c5 = + the walk-line changes) on repetitive DNA and the headline
set -uo pipefail
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -m gpu -x -q \
  --timeout 300 --timeout-method thread \
  -k "every_text or repetitive or majority or rout or verify_long or one_call or context_windows" \
  > $O/parity.log 2>&1 &&
AB_LEG=count_rdna AB_ROUNDS=2 timeout -k 10 600 bash profiles/scripts/ab_lib.sh r05t_rdna base c5 2> $O/ab1.err &&
AB_LEG=count AB_ROUNDS=2 timeout -k 10 500 bash profiles/scripts/ab_lib.sh r05t_count base c5 2> $O/ab2.err

#!/bin/bash
# r05v: list2 entries carry the chain (u32 entries, no extra array) — parity of the routed
# count and one-call locate paths, then the headline library A/B (base = the round's previous
# commit) over three rounds
set -uo pipefail
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -m gpu -x -q \
  --timeout 300 --timeout-method thread \
  -k "every_text or repetitive or majority or rout or verify_long or one_call or context_windows" \
  > $O/parity.log 2>&1 &&
AB_LEG=count AB_ROUNDS=3 timeout -k 10 600 bash profiles/scripts/ab_lib.sh r05v_count base u32 2> $O/ab.err

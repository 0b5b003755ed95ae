#!/bin/bash
# r05u: C5 (32 GB DNA) one-call locate over walk lines: full-size parity, then the library A/B
# (chain = before, c5 = barrier-free search and lockstep emit walks)
set -uo pipefail
O=gpurun_out/r05u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 500 --timeout-method thread \
  -k "c5" > $O/scale.log 2>&1 &&
AB_LEG=locate_one AB_ROUNDS=2 AB_ARGS="--text-bytes 31999999999" timeout -k 10 900 \
  bash profiles/scripts/ab_lib.sh r05u_c5_locate_one chain c5 2> $O/ab.err

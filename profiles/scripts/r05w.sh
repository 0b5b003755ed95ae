#!/bin/bash
# r05w: (1) the headline over 1, 2, 3 streams (independent batches overlapping one call's tail
# with the next call's head) and one 100 M call; (2) C5 full-size parity and the one-call
# locate library A/B (chain = before, u32 = barrier-free walk-line search + lockstep emit walks)
set -uo pipefail
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 300 python -u profiles/scripts/stream_probe.py > $O/stream_probe.json 2> $O/stream_probe.err &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 350 --timeout-method thread \
  -k "c5" > $O/scale.log 2>&1 &&
AB_LEG=locate_one AB_ROUNDS=2 AB_ARGS="--text-bytes 31999999999" timeout -k 10 700 \
  bash profiles/scripts/ab_lib.sh r05w_c5_locate_one chain u32 2> $O/ab.err

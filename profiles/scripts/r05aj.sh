#!/bin/bash
# r05aj: the one-call locate's emit over two tiles per block on full-SA indexes (e4: 4 patterns
# per lane, both tiles' records loaded before the one block scan) against a tile per block
# (head) — locate parity with e4, then the C4 locate_one A/B
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r05aj
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "locate" > $O/parity.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "c4_dna_4gb and auto" > $O/scale.log 2>&1 &&
AB_LEG=locate_one AB_ROUNDS=3 timeout -k 10 600 bash profiles/scripts/ab_lib.sh r05aj_locate_one head e4 2> $O/ab.err

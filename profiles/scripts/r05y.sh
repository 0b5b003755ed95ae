#!/bin/bash
# r05y: walk-line one-call locate with the emit's multi-position walks listed for
# k_locate_walks — parity (walk-line variants, C5 full size), the C5 kernel trace, the C5
# library A/B (chain = round-5 before, walks = now), and a C5 probe with position samples
# every 2 text positions (CS_FM_PSTRIDE=2: 80 GB of samples, if HBM allows)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r05y
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "one_call or context_windows or verify_long or every_text" > $O/parity.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 250 --timeout-method thread \
  -k "c5" > $O/scale.log 2>&1 &&
TRACE_ARGS="--text-bytes 31999999999" timeout -k 10 400 bash profiles/scripts/trace_leg.sh r05y_walks locate_one \
  > $O/trace_walks.txt 2>&1 &&
AB_LEG=locate_one AB_ROUNDS=1 AB_ARGS="--text-bytes 31999999999" timeout -k 10 500 \
  bash profiles/scripts/ab_lib.sh r05y_c5_locate_one chain walks 2> $O/ab.err &&
cp compressed-fm-index-implementation-with-learned-optimizations_amd/libcs_fmindex_walks.so \
  compressed-fm-index-implementation-with-learned-optimizations_amd/libcs_fmindex.so &&
CS_FM_PSTRIDE=2 timeout -k 10 300 python -u bench.py --only locate_one --steps 10 --warmup 2 --text-bytes 31999999999 \
  > $O/pstride2.json 2> $O/pstride2.err

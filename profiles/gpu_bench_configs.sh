#!/bin/bash
# gpu_bench_configs.sh <tag> — the bench lines of every BASELINE config in one box session
# (round 1's final numbers came from this set): C4 count-kernel profile, bench lines for
# C4 / C4 Q_unif / C4 binary wavelet / C5 / C2 / C3, the full-size property tests.
# Steps and outputs as profiles/gpu_session.sh.
TAG=${1:-final}
exec bash "$(dirname "$0")/gpu_session.sh" "$TAG" \
  "prof c4 count" "bench c4" "bench c4 --queries unif --no-cpu" \
  "bench c4 CS_FM_ENGINE=wavelet --no-cpu" "bench c5" "bench c2" "bench c3" \
  "tests test_gpu_scale"

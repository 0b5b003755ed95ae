#!/bin/bash
# gpu_profile_c4.sh — rocprofv3 passes for the default bench line (C4): kernel trace
# + stats, FETCH_SIZE, TCC hit/miss (profile_count.sh), outputs in gpurun_out/prof_<tag>.
set -e
bash profiles/profile_count.sh "${1:-c4}" > gpurun_out/prof_${1:-c4}.log 2>&1

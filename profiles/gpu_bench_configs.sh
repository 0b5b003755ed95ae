#!/bin/bash
# gpu_bench_configs.sh — the GPU-box session behind profiles/r01's numbers:
# C4 count-kernel profile (profile_count.sh), bench lines for C5 / C2 / C3, and
# the full-size property tests.  Outputs under gpurun_out/ (copied to profiles/).
set -e
bash profiles/profile_count.sh c4_occ_k14 > gpurun_out/prof_c4_occ.log 2>&1
timeout -k 10 400 python bench.py --text-bytes 31999999999 --no-cpu > gpurun_out/bench_c5_occ.json 2> gpurun_out/bench_c5_occ.err
timeout -k 10 300 python bench.py --text-bytes 99999999 --batch 1000000 > gpurun_out/bench_c2_occ.json 2> gpurun_out/bench_c2_occ.err
timeout -k 10 300 python bench.py --kind bytes --text-bytes 999999999 --m 8 --batch 10000000 > gpurun_out/bench_c3_r2.json 2> gpurun_out/bench_c3_r2.err
timeout -k 10 600 python -m pytest tests/test_gpu_scale.py -q > gpurun_out/pytest_scale3.log 2>&1

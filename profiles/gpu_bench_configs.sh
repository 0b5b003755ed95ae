#!/bin/bash
# gpu_bench_configs.sh <tag> — the GPU-box session behind profiles/r01's final numbers:
# C4 count-kernel profile (profile_count.sh: trace + FETCH_SIZE + TCC passes), bench
# lines for C4 / C4 Q_unif / C4 binary wavelet / C5 / C2 / C3, the full-size property
# tests.  Outputs under gpurun_out/ (copied to profiles/r01 by hand).
set -e
TAG=${1:-final}
bash profiles/profile_count.sh c4_$TAG > gpurun_out/prof_c4_$TAG.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err
timeout -k 10 400 python bench.py --queries unif --no-cpu > gpurun_out/bench_c4unif_$TAG.json 2> gpurun_out/bench_c4unif_$TAG.err
CS_FM_ENGINE=wavelet timeout -k 10 400 python bench.py --no-cpu > gpurun_out/bench_c4wm_$TAG.json 2> gpurun_out/bench_c4wm_$TAG.err
timeout -k 10 400 python bench.py --text-bytes 31999999999 --no-cpu > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err
timeout -k 10 300 python bench.py --text-bytes 99999999 --batch 1000000 > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err
timeout -k 10 300 python bench.py --kind bytes --text-bytes 999999999 --m 8 --batch 10000000 > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err
timeout -k 10 600 python -m pytest tests/test_gpu_scale.py -q > gpurun_out/pytest_scale_$TAG.log 2>&1

# session 2: packed wide prefix-table entries (C5 k = 16) — full GPU suite, C5 and C4 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_ptab16.log 2>&1 && \
timeout -k 10 400 python bench.py --no-cpu --host-batch 0 --text-bytes 31999999999 > gpurun_out/s2_bench_c5_ptab16.json 2> gpurun_out/s2_bench_c5_ptab16.err && \
timeout -k 10 300 python bench.py --no-cpu --host-batch 0 > gpurun_out/s2_bench_c4_ptab16.json 2> gpurun_out/s2_bench_c4_ptab16.err

# session 2: finer text-position samples — full GPU suite, C4 and C5 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_pstride.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu --host-batch 0 > gpurun_out/s2_bench_c4_pstride.json 2> gpurun_out/s2_bench_c4_pstride.err && \
timeout -k 10 400 python bench.py --no-cpu --host-batch 0 --text-bytes 31999999999 > gpurun_out/s2_bench_c5_pstride.json 2> gpurun_out/s2_bench_c5_pstride.err

# session 2: left contexts — full GPU suite, C4 bench with and without contexts
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_lctx.log 2>&1 && \
timeout -k 10 400 python bench.py --no-cpu --host-batch 0 > gpurun_out/s2_bench_c4_lctx.json 2> gpurun_out/s2_bench_c4_lctx.err && \
CS_FM_LCTX=0 timeout -k 10 400 python bench.py --no-cpu --host-batch 0 --locate-batch 0 --extract-batch 0 > gpurun_out/s2_bench_c4_nolctx.json 2> gpurun_out/s2_bench_c4_nolctx.err

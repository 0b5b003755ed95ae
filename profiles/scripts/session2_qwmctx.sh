# session 2: quaternary-matrix left contexts — full GPU suite, C3 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_qwmctx.log 2>&1 && \
timeout -k 10 300 python bench.py --kind bytes --text-bytes 999999999 --m 8 --batch 10000000 --no-cpu --host-batch 0 > gpurun_out/s2_bench_c3_ctx.json 2> gpurun_out/s2_bench_c3_ctx.err

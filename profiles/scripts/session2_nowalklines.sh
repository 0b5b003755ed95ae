# session 2: no walk lines when the full suffix array is kept — full GPU suite, C4 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_nowl.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu --host-batch 0 > gpurun_out/s2_bench_c4_nowl.json 2> gpurun_out/s2_bench_c4_nowl.err

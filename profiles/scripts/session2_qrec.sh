# session 2: quaternary-matrix context records (full GPU suite, C3 line)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2q_pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --kind bytes --text-bytes 999999999 --m 8 --batch 10000000 --no-cpu > gpurun_out/s2q_bench_c3.json 2> gpurun_out/s2q_bench_c3.err

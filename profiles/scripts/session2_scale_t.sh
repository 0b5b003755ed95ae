# session 2: full-size tests and C5 bench with the text kept in HBM
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/s2t_pytest_scale.log 2>&1 && \
timeout -k 10 400 python bench.py --text-bytes 31999999999 --no-cpu > gpurun_out/s2t_bench_c5.json 2> gpurun_out/s2t_bench_c5.err

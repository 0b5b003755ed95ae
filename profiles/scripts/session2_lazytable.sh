# session 2: node table staged only by blocks with general searches — parity subset, C2 / C4 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "count or golden or random or locate" > gpurun_out/s2_pytest_lazy.log 2>&1 && \
timeout -k 10 300 python bench.py --text-bytes 99999999 --batch 1000000 --no-cpu > gpurun_out/s2_bench_c2_lazy.json 2> gpurun_out/s2_bench_c2_lazy.err && \
timeout -k 10 300 python bench.py --no-cpu --host-batch 0 > gpurun_out/s2_bench_c4_lazy.json 2> gpurun_out/s2_bench_c4_lazy.err

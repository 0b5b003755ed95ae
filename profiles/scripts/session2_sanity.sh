set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_gpu.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/s2_bench_c4.json 2> gpurun_out/s2_bench_c4.err && \
timeout -k 10 400 python bench.py --no-cpu --prefix-k 15 --locate-batch 0 --host-batch 0 > gpurun_out/s2_bench_c4_k15.json 2> gpurun_out/s2_bench_c4_k15.err

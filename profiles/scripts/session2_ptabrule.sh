# session 2: prefix-table depth rule for large alphabets (full GPU suite, full-size tests, C3/C4 lines)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2r2_pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --kind bytes --text-bytes 999999999 --m 8 --batch 10000000 > gpurun_out/s2r2_bench_c3.json 2> gpurun_out/s2r2_bench_c3.err && \
timeout -k 10 300 python bench.py --no-cpu --host-batch 0 > gpurun_out/s2r2_bench_c4.json 2> gpurun_out/s2r2_bench_c4.err

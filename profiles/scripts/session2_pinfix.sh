# session 2: inner-page registration of caller buffers — device API tests, C2 bench line, smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_api.py tests/test_cpp_facade.py tests/test_gpu_serve.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_pinfix.log 2>&1 && \
timeout -k 10 300 python bench.py --text-bytes 99999999 --batch 1000000 > gpurun_out/s2_bench_c2_pinfix.json 2> gpurun_out/s2_bench_c2_pinfix.err && \
timeout -k 10 300 python bench.py --no-cpu --extract-batch 0 --locate-batch 0 --p50-calls 0 > gpurun_out/s2_bench_c4_pinfix.json 2> gpurun_out/s2_bench_c4_pinfix.err && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2_smoke2.log 2>&1

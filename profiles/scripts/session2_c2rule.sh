# session 2: DNA table cap n, records from k = 13 (full GPU suite, C2 and C4 lines)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2r3_pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --text-bytes 99999999 --batch 1000000 > gpurun_out/s2r3_bench_c2.json 2> gpurun_out/s2r3_bench_c2.err && \
timeout -k 10 300 python bench.py > gpurun_out/s2r3_bench_c4.json 2> gpurun_out/s2r3_bench_c4.err

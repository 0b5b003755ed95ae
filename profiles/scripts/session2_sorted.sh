# session 2: sorted-vs-random line reads microbench; C4 bench with the n/2 prefix rule
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./profiles/microbench/sorted_gather_bench 2 12.5 > gpurun_out/s2_sorted_gather.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s2_pytest_parity.log 2>&1 && \
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/s2_bench_c4_auto.json 2> gpurun_out/s2_bench_c4_auto.err

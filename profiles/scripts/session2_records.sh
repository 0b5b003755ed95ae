# session 2: context records — full GPU suite, C4 bench with and without records
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_records.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu --host-batch 0 > gpurun_out/s2_bench_c4_records.json 2> gpurun_out/s2_bench_c4_records.err && \
CS_FM_CTX_RECORDS=0 timeout -k 10 300 python bench.py --no-cpu --host-batch 0 --extract-batch 0 --locate-batch 0 > gpurun_out/s2_bench_c4_norec.json 2> gpurun_out/s2_bench_c4_norec.err

# session 2: fixed-length count entry point (parity + C4 bench line)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fixed_length or engine_choice" > gpurun_out/s2x_pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu --host-batch 0 --locate-batch 0 --extract-batch 0 > gpurun_out/s2x_bench_c4.json 2> gpurun_out/s2x_bench_c4.err

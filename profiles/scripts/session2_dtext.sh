# session 2: text in HBM for extract (parity + C4 bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2t_pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu --host-batch 0 > gpurun_out/s2t_bench_c4.json 2> gpurun_out/s2t_bench_c4.err && \
CS_FM_DEVICE_TEXT=0 timeout -k 10 300 python bench.py --no-cpu --host-batch 0 --locate-batch 0 > gpurun_out/s2t_bench_c4_lf.json 2> gpurun_out/s2t_bench_c4_lf.err

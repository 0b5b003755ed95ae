# session 2: compact 16-B context records (parity, device API, C4 count vs 32-B records)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rec or engine_choice or export_import" > gpurun_out/s2r_pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu --host-batch 0 --extract-batch 0 > gpurun_out/s2r_bench_c4_rec16.json 2> gpurun_out/s2r_bench_c4_rec16.err && \
CS_FM_CTX_RECORDS=1 timeout -k 10 300 python bench.py --no-cpu --host-batch 0 --extract-batch 0 > gpurun_out/s2r_bench_c4_rec32.json 2> gpurun_out/s2r_bench_c4_rec32.err && \
timeout -k 10 300 python bench.py --no-cpu --host-batch 0 --extract-batch 0 --queries unif > gpurun_out/s2r_bench_c4u_rec16.json 2> gpurun_out/s2r_bench_c4u_rec16.err

# session 2: fused full-SA locate phase 2 (parity, full-size tests, C4 locate line)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -m gpu -x -q --timeout 300 --timeout-method thread -k "locate or every_text or golden or create or save" > gpurun_out/s2l_pytest.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c4_dna_4gb and auto or c2 or c3" > gpurun_out/s2l_pytest_scale.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu --host-batch 0 --extract-batch 0 > gpurun_out/s2l_bench_c4.json 2> gpurun_out/s2l_bench_c4.err

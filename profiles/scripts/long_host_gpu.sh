set -o pipefail
mkdir -p gpurun_out/longhost
timeout -k 10 900 python -u -m pytest tests/test_gpu_device_api.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "device_api or verify_long" > gpurun_out/longhost/pytest.log 2>&1 || { tail -40 gpurun_out/longhost/pytest.log; exit 1; }
tail -2 gpurun_out/longhost/pytest.log
timeout -k 10 150 python -u bench.py --only count > gpurun_out/longhost/count.json 2> gpurun_out/longhost/count.err || exit 1
timeout -k 10 150 python -u bench.py --only host_batch > gpurun_out/longhost/host_batch.json 2> gpurun_out/longhost/host_batch.err || exit 1

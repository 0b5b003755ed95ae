# session 2: device API tests (export/import with records and full SA)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_device_api.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_devapi.log 2>&1

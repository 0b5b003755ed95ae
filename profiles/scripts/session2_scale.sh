# session 2: full-size property tests (C2-C5) with the C4 index variants
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/s2_pytest_scale_variants.log 2>&1

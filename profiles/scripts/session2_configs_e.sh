# session 2e: full GPU suite, then the config benches + C4 count profile with compact records
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2e_pytest_gpu.log 2>&1 && \
bash profiles/gpu_bench_configs.sh s2e

# session 2: final verification (GPU suite, smoke, default bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2f_pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s2f_smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/s2f_bench.json 2> gpurun_out/s2f_bench.err

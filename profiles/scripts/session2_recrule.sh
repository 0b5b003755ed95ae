# session 2: records from 14-character tables — full GPU suite, C2 bench line, smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_recrule.log 2>&1 && \
timeout -k 10 300 python bench.py --text-bytes 99999999 --batch 1000000 > gpurun_out/s2_bench_c2_recrule.json 2> gpurun_out/s2_bench_c2_recrule.err && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2_smoke2.log 2>&1

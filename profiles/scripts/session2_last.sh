# session 2: last check of the final tree (smoke, default bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s2last_smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/s2last_bench.json 2> gpurun_out/s2last_bench.err

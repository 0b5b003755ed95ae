# session 2: staged context count kernel — GPU suite, then C4 count with U = 1, 2, 4 patterns per lane
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_countu.log 2>&1 && \
for u in 1 2 4; do
  CS_FM_COUNT_U=$u timeout -k 10 300 python bench.py --no-cpu --host-batch 0 --locate-batch 0 --extract-batch 0 > gpurun_out/s2_bench_c4_u$u.json 2> gpurun_out/s2_bench_c4_u$u.err || exit 1
done

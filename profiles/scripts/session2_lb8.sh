# session 2: count kernels at 8 waves/SIMD (launch bounds) — C4 count with U = 1, 2
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "count_every or golden or random" > gpurun_out/s2_pytest_lb8.log 2>&1 && \
for u in 1 2; do
  CS_FM_COUNT_U=$u timeout -k 10 300 python bench.py --no-cpu --host-batch 0 --extract-batch 0 --p50-calls 0 > gpurun_out/s2_bench_c4_lb8_u$u.json 2> gpurun_out/s2_bench_c4_lb8_u$u.err || exit 1
done

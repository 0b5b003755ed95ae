# session 2: staged kernels with a 512-B LDS code map — parity subset, C4 count with U = 1, 2
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "count or golden or random or locate" > gpurun_out/s2_pytest_cmap.log 2>&1 && \
for u in 2 1; do
  CS_FM_COUNT_U=$u timeout -k 10 300 python bench.py --no-cpu --host-batch 0 --extract-batch 0 > gpurun_out/s2_bench_c4_cmap_u$u.json 2> gpurun_out/s2_bench_c4_cmap_u$u.err || exit 1
done

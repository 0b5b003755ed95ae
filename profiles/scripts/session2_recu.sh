# session 2: context records — C4 count with U = 1, 2, 4 patterns per lane
set -o pipefail
cd $GRAFT_REPO_ROOT
for u in 1 2 4; do
  CS_FM_COUNT_U=$u timeout -k 10 300 python bench.py --no-cpu --host-batch 0 --extract-batch 0 --locate-batch 0 --p50-calls 0 > gpurun_out/s2_bench_c4_rec_u$u.json 2> gpurun_out/s2_bench_c4_rec_u$u.err || exit 1
done

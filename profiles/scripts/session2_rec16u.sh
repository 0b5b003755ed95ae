# session 2: compact records, patterns per lane sweep (is the count kernel latency-bound?)
set -o pipefail
cd $GRAFT_REPO_ROOT
for u in 1 4; do
  CS_FM_COUNT_U=$u timeout -k 10 300 python bench.py --no-cpu --host-batch 0 --locate-batch 0 --extract-batch 0 > gpurun_out/s2r_bench_c4_rec16_u$u.json 2> gpurun_out/s2r_bench_c4_rec16_u$u.err || exit 1
done

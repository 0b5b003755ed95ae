# session 2: C4 with a k = 16 table (compact records over 69 GB)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --no-cpu --host-batch 0 --extract-batch 0 --prefix-k 16 > gpurun_out/s2k16_bench_c4.json 2> gpurun_out/s2k16_bench_c4.err

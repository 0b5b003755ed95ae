# session 2: C3 (sigma = 256) with a deeper prefix table (k = 4: 2^32 entries, 34 GB)
set -o pipefail
cd $GRAFT_REPO_ROOT
CS_FM_VERBOSE=1 timeout -k 10 400 python bench.py --kind bytes --text-bytes 999999999 --m 8 --batch 10000000 --no-cpu --prefix-k 4 > gpurun_out/s2k_bench_c3_k4.json 2> gpurun_out/s2k_bench_c3_k4.err

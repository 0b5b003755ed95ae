# session 2: C2 (100 MB DNA) with a k = 13 table, without and with 32-B context records
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench.py --text-bytes 99999999 --batch 1000000 --no-cpu --prefix-k 13 > gpurun_out/s2c2_k13.json 2> gpurun_out/s2c2_k13.err && \
CS_FM_CTX_RECORDS=1 timeout -k 10 200 python bench.py --text-bytes 99999999 --batch 1000000 --no-cpu --prefix-k 13 > gpurun_out/s2c2_k13_rec.json 2> gpurun_out/s2c2_k13_rec.err && \
timeout -k 10 200 python bench.py --text-bytes 99999999 --batch 1000000 --no-cpu > gpurun_out/s2c2_k12.json 2> gpurun_out/s2c2_k12.err

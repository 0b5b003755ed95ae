# session 2: build phase timings (records vs none)
set -o pipefail
cd $GRAFT_REPO_ROOT
CS_FM_VERBOSE=1 timeout -k 10 300 python bench.py --no-cpu --host-batch 0 --locate-batch 0 --extract-batch 0 --steps 5 > gpurun_out/s2b_rec16.json 2> gpurun_out/s2b_rec16.err && \
CS_FM_VERBOSE=1 CS_FM_CTX_RECORDS=0 timeout -k 10 300 python bench.py --no-cpu --host-batch 0 --locate-batch 0 --extract-batch 0 --steps 5 > gpurun_out/s2b_rec0.json 2> gpurun_out/s2b_rec0.err

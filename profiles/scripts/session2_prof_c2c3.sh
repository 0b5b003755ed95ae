# session 2: count-kernel profiles (trace + FETCH_SIZE + TCC) of C2 and C3
set -o pipefail
cd $GRAFT_REPO_ROOT
bash profiles/profile_count.sh c2_s2e3 --text-bytes 99999999 --batch 1000000 --locate-batch 0 --extract-batch 0 --host-batch 0 > gpurun_out/prof_c2_s2e3.log 2>&1 && \
bash profiles/profile_count.sh c3_s2e3 --kind bytes --text-bytes 999999999 --m 8 --batch 10000000 --locate-batch 0 --extract-batch 0 --host-batch 0 > gpurun_out/prof_c3_s2e3.log 2>&1

# session 2: locate phase 1 with one vs two patterns per lane
set -o pipefail
cd $GRAFT_REPO_ROOT
CS_FM_LOCATE_U=1 timeout -k 10 200 python profiles/scripts/locate_phases.py > gpurun_out/s2u_locate_u1.json 2> gpurun_out/s2u_locate_u1.err && \
timeout -k 10 200 python profiles/scripts/locate_phases.py > gpurun_out/s2u_locate_u2.json 2> gpurun_out/s2u_locate_u2.err

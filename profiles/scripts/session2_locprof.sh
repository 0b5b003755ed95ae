# session 2: C4 locate phases and their kernels (rocprofv3 kernel trace)
set -o pipefail
cd $GRAFT_REPO_ROOT
python profiles/scripts/locate_phases.py > gpurun_out/s2p_locate_phases.json 2> gpurun_out/s2p_locate_phases.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/s2p_locprof -o run -- python3 $GRAFT_REPO_ROOT/profiles/scripts/locate_phases.py > $GRAFT_REPO_ROOT/gpurun_out/s2p_locate_phases_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/s2p_locprof.err

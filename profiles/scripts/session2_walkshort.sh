# session 2: one-lane-per-row walk for position-marked walk lines vs the persistent walk
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_walkshort.log 2>&1 && \
timeout -k 10 300 python profiles/scripts/locate_phases.py > gpurun_out/s2_locate_phases_short.json 2> gpurun_out/s2_locate_phases_short.err && \
CS_FM_WALK_PERSISTENT=1 timeout -k 10 300 python profiles/scripts/locate_phases.py > gpurun_out/s2_locate_phases_persist.json 2> gpurun_out/s2_locate_phases_persist.err && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2_smoke.log 2>&1

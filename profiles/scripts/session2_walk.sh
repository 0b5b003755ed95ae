# session 2: walk with the next row fetched beside the sample; position stride 8 vs 4
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -m gpu -x -q --timeout 300 --timeout-method thread -k "locate or walk or device or golden or strides or bucketed or random" > gpurun_out/s2_pytest_walk.log 2>&1 && \
timeout -k 10 300 python profiles/scripts/locate_phases.py > gpurun_out/s2_locate_phases_merge.json 2> gpurun_out/s2_locate_phases_merge.err && \
CS_FM_PSTRIDE=4 timeout -k 10 300 python profiles/scripts/locate_phases.py > gpurun_out/s2_locate_phases_p4.json 2> gpurun_out/s2_locate_phases_p4.err

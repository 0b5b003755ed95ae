# session 2: short walk without the LDS node table
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "locate or golden or strides or random" > gpurun_out/s2_pytest_walknolds.log 2>&1 && \
timeout -k 10 300 python profiles/scripts/locate_phases.py > gpurun_out/s2_locate_phases_nolds.json 2> gpurun_out/s2_locate_phases_nolds.err

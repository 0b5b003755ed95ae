# session 2: parity of the one-pattern-per-lane kernels (auto_rec16 variant) + 2-rank rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "auto_rec16" > gpurun_out/s2c_pytest.log 2>&1 && \
bash profiles/scripts/session2_rehearse2.sh

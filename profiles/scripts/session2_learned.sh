# session 2: learned occurrence lines — full GPU suite, C4 bench on the learned engine
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_learned.log 2>&1 && \
CS_FM_ENGINE=learned timeout -k 10 300 python bench.py --no-cpu --host-batch 0 > gpurun_out/s2_bench_c4_learned.json 2> gpurun_out/s2_bench_c4_learned.err

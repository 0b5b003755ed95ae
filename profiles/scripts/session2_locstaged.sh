# session 2: staged locate phase 1 — full GPU suite, locate phases, C4 bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_locstaged.log 2>&1 && \
timeout -k 10 300 python profiles/scripts/locate_phases.py > gpurun_out/s2_locate_phases_staged.json 2> gpurun_out/s2_locate_phases_staged.err && \
timeout -k 10 300 python bench.py --no-cpu --host-batch 0 > gpurun_out/s2_bench_c4_locstaged.json 2> gpurun_out/s2_bench_c4_locstaged.err

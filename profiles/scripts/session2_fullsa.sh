# session 2: locate through the full suffix array — full GPU suite, locate phases, C4 / C3 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_fullsa.log 2>&1 && \
timeout -k 10 300 python profiles/scripts/locate_phases.py > gpurun_out/s2_locate_phases_fullsa.json 2> gpurun_out/s2_locate_phases_fullsa.err && \
timeout -k 10 300 python bench.py --no-cpu --host-batch 0 > gpurun_out/s2_bench_c4_fullsa.json 2> gpurun_out/s2_bench_c4_fullsa.err && \
timeout -k 10 300 python bench.py --kind bytes --text-bytes 999999999 --m 8 --batch 10000000 --no-cpu --host-batch 0 > gpurun_out/s2_bench_c3_fullsa.json 2> gpurun_out/s2_bench_c3_fullsa.err

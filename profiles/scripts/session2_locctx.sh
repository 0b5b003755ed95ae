# session 2: locate ranges over context windows — full GPU suite, C4 / C3 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_pytest_locctx.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu --host-batch 0 > gpurun_out/s2_bench_c4_locctx.json 2> gpurun_out/s2_bench_c4_locctx.err && \
timeout -k 10 300 python bench.py --kind bytes --text-bytes 999999999 --m 8 --batch 10000000 --no-cpu --host-batch 0 > gpurun_out/s2_bench_c3_locctx.json 2> gpurun_out/s2_bench_c3_locctx.err && \
timeout -k 10 300 python profiles/scripts/locate_phases.py > gpurun_out/s2_locate_phases.json 2> gpurun_out/s2_locate_phases.err

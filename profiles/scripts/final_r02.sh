#!/bin/bash
# round-2 closing run on one GPU: PMC/kernel stats of the long-pattern legs, the full
# GPU suite, smoke, the default bench line
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out/final
bash profiles/profile_legs.sh r02L count_m150_long,count_m64_long > gpurun_out/final/prof.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/final/prof.log; exit 1; }
echo "profiles done"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/final/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/final/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { cat gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 700 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail -20 gpurun_out/final/bench.err; exit 1; }
echo "bench done"

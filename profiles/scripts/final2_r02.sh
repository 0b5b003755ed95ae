#!/bin/bash
# round-2 closing check of the final tree: the full GPU suite and smoke
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out/final2
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final2/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/final2/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/final2/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2/smoke.log 2>&1 || { cat gpurun_out/final2/smoke.log; exit 1; }
tail -1 gpurun_out/final2/smoke.log

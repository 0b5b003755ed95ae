#!/bin/bash
# r05ah: the round's closing check on one box — the whole -m gpu suite as the driver runs it,
# smoke(), then bench.py's default line (N = 1)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r05ah
mkdir -p $O
cd $R
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=25 \
  > $O/pytest_gpu_all.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err

#!/bin/bash
# the whole -m gpu suite (as the driver runs it), timed, with the slowest tests listed
set -uo pipefail
O=gpurun_out/${TAG:-r05_suite}
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=40 \
  > $O/pytest_gpu_all.log 2>&1
rc=$?
tail -50 $O/pytest_gpu_all.log
exit $rc

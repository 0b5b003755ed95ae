#!/bin/bash
# round 5, first GPU session: parity subset over the routed-by-default path, then the C4
# headline with the new legs (workspace, 100 M batch, repetitive DNA with listed general
# searches, one-call locate with the workspace)
set -uo pipefail
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -x -q \
  --timeout 120 --timeout-method thread -m gpu \
  -k "((long or locate_records or repetitive or majority or every_text or widths or verify) and auto and not auto_) or device_api or learned-rep" \
  > $O/pytest_subset.log 2>&1 || { tail -30 $O/pytest_subset.log; exit 1; }
tail -3 $O/pytest_subset.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --legs count_100m,count_rdna,locate_one,count_m150,count_m150_staged \
  --legs-out $O/bench_full.json > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json

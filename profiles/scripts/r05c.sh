#!/bin/bash
# round 5: parity subset after the per-wave general-list threshold, then the threshold A/B
# (CS_FM_GENERAL_LIST_MIN, read at build) on the headline and the repetitive-DNA leg
set -uo pipefail
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -x -q \
  --timeout 120 --timeout-method thread -m gpu \
  -k "((long or locate_records or repetitive or majority or every_text or widths or verify) and auto and not auto_) or device_api or learned-rep" \
  > $O/pytest_subset.log 2>&1 || { tail -30 $O/pytest_subset.log; exit 1; }
tail -2 $O/pytest_subset.log
for T in 4 2 8 1; do
  CS_FM_GENERAL_LIST_MIN=$T timeout -k 10 200 python -u bench.py --only count --steps 30 --warmup 5 > $O/count_t$T.json 2> $O/count_t$T.err || exit 1
  CS_FM_GENERAL_LIST_MIN=$T timeout -k 10 200 python -u bench.py --only count_rdna --steps 30 --warmup 5 > $O/rdna_t$T.json 2> $O/rdna_t$T.err || exit 1
  python3 -c "
import json
c=json.load(open('$O/count_t$T.json'))['count']; r=json.load(open('$O/rdna_t$T.json'))['legs']['count_rdna']
print('T=$T count %.4f ms  rdna %.4f ms' % (c['kernel_ms_median'], r['kernel_ms_mean']))"
done

#!/bin/bash
# round 5: parity subset after the lockstep list stepper (ranges passed through the
# workspace), then the headline, repetitive DNA and 150-mer legs
set -uo pipefail
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -x -q \
  --timeout 120 --timeout-method thread -m gpu \
  -k "((long or locate_records or repetitive or majority or every_text or widths or verify) and auto and not auto_) or device_api or learned-rep or wide_rec16-rep or qwm-rep" \
  > $O/pytest_subset.log 2>&1 || { tail -30 $O/pytest_subset.log; exit 1; }
tail -2 $O/pytest_subset.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --legs count_rdna,count_m150,count_m64,locate_one,count_100m \
  --legs-out $O/bench_full.json > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d=json.load(open('gpurun_out/r05d/bench_full.json'))
print('headline', d['ms_per_step'], d['roofline']['kernel_ms_median'])
for k,v in d['legs'].items():
    print(k, v.get('kernel_ms_mean') or v.get('event_ms'), v.get('patterns_per_s'))
PY

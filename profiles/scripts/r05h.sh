#!/bin/bash
# round 5: parity after the emit-side look-back scan (one-call locate: two launches), then
# the locate and list legs
set -uo pipefail
O=gpurun_out/${TAG:-r05h}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -x -q \
  --timeout 120 --timeout-method thread -m gpu \
  -k "((long or locate or repetitive or majority or every_text or widths or verify or golden) and (auto- or auto_nosa or wide_rec16- or learned- or qwm-)) or device_api" \
  > $O/pytest_subset.log 2>&1 || { tail -40 $O/pytest_subset.log; exit 1; }
tail -2 $O/pytest_subset.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --legs count_rdna,count_m150,count_m64,locate_one,locate_m64,locate_m150,locate \
  --legs-out $O/bench_full.json > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d=json.load(open('gpurun_out/'+__import__("os").environ.get("TAG","r05h")+'/bench_full.json'))
print('headline', d['ms_per_step'], d['roofline']['kernel_ms_median'])
for k,v in d['legs'].items():
    print(k, v.get('kernel_ms_mean') or v.get('event_ms'), v.get('seconds'), v.get('patterns_per_s'), v.get('positions_verified'))
PY

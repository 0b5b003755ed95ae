set -uo pipefail
O=gpurun_out/r04i
mkdir -p $O
P=profiles/scripts/ab_probe.py
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_api.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "locate or long or rout or null" > $O/parity.log 2>&1 &&
timeout -k 10 300 python -u $P --rounds 4 --b2b --reps 20 --hook CS_FM_LONG_ROUTE=0 > $O/ab_route.json 2> $O/ab_route.err &&
timeout -k 10 300 python -u $P --rounds 4 --b2b --reps 20 --hook CS_FM_COUNT_NOBAR=0 > $O/ab_nobar.json 2> $O/ab_nobar.err &&
timeout -k 10 300 python -u $P --op locate --rounds 4 --reps 5 --hook CS_FM_LOC_DEFER=1 > $O/ab_defer.json 2> $O/ab_defer.err &&
timeout -k 10 300 python -u bench.py --only locate_m150 --steps 10 --warmup 2 > $O/locate_m150.json 2> $O/locate_m150.err &&
timeout -k 10 300 python -u bench.py --only count_m150 --steps 10 --warmup 2 > $O/count_m150.json 2> $O/count_m150.err

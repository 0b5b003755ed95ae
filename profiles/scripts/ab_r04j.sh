set -uo pipefail
O=gpurun_out/r04j
mkdir -p $O
P=profiles/scripts/ab_probe.py
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_api.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "locate or long or rout or null" > $O/parity.log 2>&1 &&
timeout -k 10 300 python -u $P --rounds 4 --b2b --reps 20 --hook CS_FM_LONG_ROUTE=0 > $O/ab_route.json 2> $O/ab_route.err &&
AB_LEG=count_m150 AB_ROUNDS=2 timeout -k 10 400 bash profiles/scripts/ab_lib.sh r04j_count_m150 base w4 2> $O/ab_lib1.err &&
AB_LEG=locate_m150 AB_ROUNDS=2 timeout -k 10 400 bash profiles/scripts/ab_lib.sh r04j_locate_m150 base w4 2> $O/ab_lib2.err

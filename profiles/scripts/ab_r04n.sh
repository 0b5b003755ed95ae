set -uo pipefail
O=gpurun_out/r04n
mkdir -p $O
P=profiles/scripts/ab_probe.py
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_api.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "locate or long or rout or null" > $O/parity.log 2>&1 &&
timeout -k 10 300 python -u $P --op locate --rounds 4 --reps 5 --hook CS_FM_COUNT_NOBAR=0 > $O/ab_loc_nobar.json 2> $O/ab_loc_nobar.err &&
AB_LEG=locate_one AB_ROUNDS=2 timeout -k 10 500 bash profiles/scripts/ab_lib.sh r04n_locate_one base w6 2> $O/ab_lib.err &&
bash profiles/scripts/ab_r04m.sh

set -uo pipefail
mkdir -p gpurun_out/r04f
P=profiles/scripts/ab_probe.py
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04f/parity.log 2>&1 &&
timeout -k 10 300 python -u $P --rounds 4 --hook CS_FM_COUNT_NOBAR=0 > gpurun_out/r04f/ab_nobar.json 2> gpurun_out/r04f/ab_nobar.err &&
timeout -k 10 300 python -u $P --op locate --rounds 4 --reps 5 --hook CS_FM_LOC_DEFER=0 > gpurun_out/r04f/ab_defer.json 2> gpurun_out/r04f/ab_defer.err

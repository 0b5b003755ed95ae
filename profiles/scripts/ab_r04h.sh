set -uo pipefail
mkdir -p gpurun_out/r04h
P=profiles/scripts/ab_probe.py
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_api.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "locate or long or rout" > gpurun_out/r04h/parity.log 2>&1 &&
timeout -k 10 300 python -u $P --rounds 4 --hook CS_FM_LONG_ROUTE=0 > gpurun_out/r04h/ab_route.json 2> gpurun_out/r04h/ab_route.err &&
timeout -k 10 300 python -u bench.py --only locate_m150 --steps 10 --warmup 2 > gpurun_out/r04h/locate_m150.json 2> gpurun_out/r04h/locate_m150.err &&
timeout -k 10 300 python -u bench.py --only count_m150 --steps 10 --warmup 2 > gpurun_out/r04h/count_m150.json 2> gpurun_out/r04h/count_m150.err

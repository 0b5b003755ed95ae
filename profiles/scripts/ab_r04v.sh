set -uo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_api.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "locate or rout or null" > $O/parity.log 2>&1 &&
timeout -k 10 300 python -u profiles/scripts/ab_probe.py --op locate --rounds 3 --reps 5 --hook CS_FM_LOC_DEFER=1 > $O/ab64.json 2> $O/ab64.err &&
CS_FM_LOC_REC64=0 timeout -k 10 300 python -u profiles/scripts/ab_probe.py --op locate --rounds 3 --reps 5 --hook CS_FM_LOC_DEFER=1 > $O/ab16.json 2> $O/ab16.err &&
timeout -k 10 300 python -u bench.py --only locate_one --steps 10 --warmup 2 > $O/locate_one64.json 2> $O/locate_one64.err &&
CS_FM_LOC_REC64=0 timeout -k 10 300 python -u bench.py --only locate_one --steps 10 --warmup 2 > $O/locate_one16.json 2> $O/locate_one16.err

set -uo pipefail
O=gpurun_out/r04ac
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "locate" > $O/parity.log 2>&1 &&
timeout -k 10 400 python -u bench.py --text-bytes 31999999999 --only locate_one --steps 5 --warmup 1 > $O/c5_pair.json 2> $O/c5_pair.err &&
CS_FM_WALK_PAIR=0 timeout -k 10 400 python -u bench.py --text-bytes 31999999999 --only locate_one --steps 5 --warmup 1 > $O/c5_nopair.json 2> $O/c5_nopair.err

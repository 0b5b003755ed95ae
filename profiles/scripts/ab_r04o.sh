set -uo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_api.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "locate or long or rout or null" > $O/parity.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_loc -o run -- python3 $GRAFT_REPO_ROOT/profiles/scripts/ab_probe.py --op locate --rounds 1 --reps 5 > $O/ab_loc.json 2> $O/ab_loc.err

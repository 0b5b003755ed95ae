set -uo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "locate_records or locate_one or locate_verify" > $O/parity.log 2>&1 &&
timeout -k 10 300 python -u profiles/scripts/ab_probe.py --op locate --rounds 4 --reps 5 --hook CS_FM_LOC_DEFER=1 > $O/ab_defer.json 2> $O/ab_defer.err &&
cd /tmp && export TMPDIR=/tmp &&
CS_FM_LOC_DEFER=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_def -o run -- python3 $GRAFT_REPO_ROOT/profiles/scripts/ab_probe.py --op locate --rounds 1 --reps 5 > $O/ab_def.json 2> $O/ab_def.err

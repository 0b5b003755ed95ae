set -uo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CS_FM_LOC_DEFER=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_def -o run -- python3 $GRAFT_REPO_ROOT/profiles/scripts/ab_probe.py --op locate --rounds 1 --reps 5 > $O/ab_def.json 2> $O/ab_def.err &&
cd $GRAFT_REPO_ROOT && timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -v --timeout 600 --timeout-method thread > $O/scale.log 2>&1

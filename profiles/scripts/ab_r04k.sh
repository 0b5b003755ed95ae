set -uo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04k
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/profiles/scripts/ab_probe.py --rounds 1 --b2b --reps 10 --hook CS_FM_LONG_ROUTE=0 > $O/ab.json 2> $O/ab.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_loc -o run -- python3 $GRAFT_REPO_ROOT/profiles/scripts/ab_probe.py --op locate --rounds 1 --reps 5 --hook CS_FM_LONG_ROUTE=0 > $O/ab_loc.json 2> $O/ab_loc.err

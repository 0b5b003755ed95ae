#!/bin/bash
# round 5 measurement session 1: routing A/Bs back to back (the staged kernel alone vs routed
# with the workspace vs routed with the per-call allocation) at C4 and C2, then the headline's
# rocprofv3 passes over 30 timed launches (kernel trace, FETCH_SIZE, L2)
set -uo pipefail
O=gpurun_out/r05p
mkdir -p $O
P=profiles/scripts/ab_probe.py
timeout -k 10 300 python -u $P --b2b --flags-a NO_ROUTE --flags-b "" --ws-b > $O/ab_route_c4.json 2> $O/ab_route_c4.err || exit 1
timeout -k 10 300 python -u $P --b2b --flags-a "" --flags-b "" --ws-b > $O/ab_ws_c4.json 2> $O/ab_ws_c4.err || exit 1
timeout -k 10 300 python -u $P --b2b --text-bytes 99999999 --batch 1000000 --reps 50 --flags-a NO_ROUTE --flags-b "" --ws-b \
  > $O/ab_route_c2.json 2> $O/ab_route_c2.err || exit 1
timeout -k 10 300 python -u $P --b2b --text-bytes 99999999 --batch 1000000 --reps 50 --flags-a "" --flags-b "" --ws-b \
  > $O/ab_ws_c2.json 2> $O/ab_ws_c2.err || exit 1
grep -h "\[ab\]" $O/*.err
PROF_STEPS=30 PROF_WARMUP=5 timeout -k 10 900 bash profiles/profile_legs.sh r05p_c4 count > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -12 $O/prof.log

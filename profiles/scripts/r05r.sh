#!/bin/bash
# round 5 measurement session: the C4 line (every leg), the C2 and C3 lines, and the C2 count's
# rocprofv3 passes (FETCH_SIZE at C2)
set -uo pipefail
timeout -k 10 1100 bash profiles/gpu_session.sh r05r "bench c4" "bench c2" "bench c3" "prof c2 count" > gpurun_out/r05r_session.log 2>&1
rc=$?
tail -5 gpurun_out/r05r_session.log
for f in gpurun_out/r05r_*_bench_*.json; do echo "$f"; cut -c1-400 "$f"; done
exit $rc

#!/bin/bash
# round 5: kernel trace of the routed headline, general searches listed (default) vs in the
# lane (CS_FM_GENERAL_INLANE=1 at build), and of the repetitive-DNA leg the same two ways
set -uo pipefail
O=$PWD/gpurun_out/${TAG:-r05b}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in list inlane; do
  if [ $v = inlane ]; then export CS_FM_GENERAL_INLANE=1; else unset CS_FM_GENERAL_INLANE; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- \
    python3 $R/bench.py --only count --steps 30 --warmup 5 > $O/count_$v.json 2> $O/count_$v.err || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_rdna_$v -o run -- \
    python3 $R/bench.py --only count_rdna --steps 30 --warmup 5 > $O/rdna_$v.json 2> $O/rdna_$v.err || exit 1
done
python3 $R/profiles/summarize.py $O/trace_list r05b_list > /dev/null 2>&1 || true
for d in $O/trace_*; do
  echo "== $d"
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  head -6 "$f" | cut -c1-220
done

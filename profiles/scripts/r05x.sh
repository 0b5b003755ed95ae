#!/bin/bash
# r05x: C5 one-call locate kernel traces with the library before (chain) and after (u32) the
# walk-line changes, then the stream probe with more rounds
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
PKG=$R/compressed-fm-index-implementation-with-learned-optimizations_amd
O=$R/gpurun_out/r05x
mkdir -p $O
cp $PKG/libcs_fmindex.so $PKG/libcs_fmindex_cur.so
for V in chain u32; do
  cp $PKG/libcs_fmindex_$V.so $PKG/libcs_fmindex.so
  TRACE_ARGS="--text-bytes 31999999999" timeout -k 10 400 bash $R/profiles/scripts/trace_leg.sh r05x_$V locate_one \
    > $O/trace_$V.txt 2>&1 || exit 1
done
cp $PKG/libcs_fmindex_cur.so $PKG/libcs_fmindex.so
cd $R && timeout -k 10 400 python -u profiles/scripts/stream_probe.py --streams 1,2,3,4 --rounds 7 \
  > $O/stream_probe.json 2> $O/stream_probe.err

#!/bin/bash
# round 5: the list kernels' grid (CS_FM_LIST_GRID, read at build) against the legs that
# list: repetitive DNA (general searches), 150- and 64-mers (long patterns), 150-mer locate
set -uo pipefail
O=gpurun_out/${TAG:-r05f}
mkdir -p $O
for G in ${GRIDS:-2560 1024 4096}; do
  for L in ${LEGS:-count_rdna count_m150 count_m64 locate_m150}; do
    CS_FM_LIST_GRID=$G timeout -k 10 200 python -u bench.py --only $L --steps 20 --warmup 3 > $O/${L}_g$G.json 2> $O/${L}_g$G.err || exit 1
    python3 -c "
import json
l=json.load(open('$O/${L}_g$G.json'))['legs']['$L']
print('G=$G $L', l.get('kernel_ms_mean') or l.get('event_ms'))"
  done
done

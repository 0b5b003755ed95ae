#!/bin/bash
# r05am: the routed list kernel's grid (CS_FM_LIST_GRID, read at handle creation; default 4
# blocks per CU = 1024) — the headline (an empty list kernel: its dispatch is the cost) and
# 150-mers (a full list) at 512 / 1024 / 2048 blocks, two rounds, a process per run
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r05am
mkdir -p $O
cd $R
: > $O/grid.jsonl
for round in 1 2; do
  for leg in count count_m150; do
    for g in 512 1024 2048; do
      r=$(CS_FM_LIST_GRID=$g timeout -k 10 240 python3 bench.py --only $leg --steps 30 --warmup 5 | tail -1) || exit 1
      echo "{\"grid\": $g, \"leg\": \"$leg\", \"round\": $round, \"result\": $r}" >> $O/grid.jsonl
    done
  done
done

set -uo pipefail
O=gpurun_out/r04y
mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --only count_packed --steps 30 --warmup 5 > $O/packed_u2_$r.json 2> $O/packed_u2_$r.err || exit 1
  CS_FM_COUNT_U=4 timeout -k 10 300 python -u bench.py --only count_packed --steps 30 --warmup 5 > $O/packed_u4_$r.json 2> $O/packed_u4_$r.err || exit 1
done

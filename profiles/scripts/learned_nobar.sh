mkdir -p gpurun_out/lnb
for nb in 0 1; do
  CS_FM_COUNT_NOBAR=$nb timeout -k 10 150 python -u bench.py --only learned_count > gpurun_out/lnb/learned_nb$nb.json 2> gpurun_out/lnb/learned_nb$nb.err || exit 1
  CS_FM_COUNT_NOBAR=$nb timeout -k 10 150 python -u bench.py --only count > gpurun_out/lnb/count_nb$nb.json 2> gpurun_out/lnb/count_nb$nb.err || exit 1
done

set -uo pipefail
mkdir -p gpurun_out/r04e
P=profiles/scripts/ab_probe.py
timeout -k 10 300 python -u $P --rounds 4 --hook CS_FM_LONG_ROUTE=0 > gpurun_out/r04e/ab_route.json 2> gpurun_out/r04e/ab_route.err &&
timeout -k 10 300 python -u $P --rounds 4 --hook CS_FM_COUNT_NOBAR=1 > gpurun_out/r04e/ab_nobar.json 2> gpurun_out/r04e/ab_nobar.err &&
timeout -k 10 300 python -u $P --op locate --rounds 4 --reps 5 --hook CS_FM_LOC_DEFER=0 > gpurun_out/r04e/ab_defer.json 2> gpurun_out/r04e/ab_defer.err &&
CS_FM_LOC_RECORDS=0 timeout -k 10 300 python -u $P --rounds 3 --hook CS_FM_LONG_ROUTE=0 > gpurun_out/r04e/ab_nolrec.json 2> gpurun_out/r04e/ab_nolrec.err

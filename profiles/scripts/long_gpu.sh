set -o pipefail
mkdir -p gpurun_out/long
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "verify_long or query_flags_count or count_ex" > gpurun_out/long/pytest.log 2>&1 || { tail -30 gpurun_out/long/pytest.log; exit 1; }
tail -3 gpurun_out/long/pytest.log
for leg in count_m150_long count_m64_long count_m150 count_m64; do
  timeout -k 10 150 python -u bench.py --only $leg > gpurun_out/long/$leg.json 2> gpurun_out/long/$leg.err || exit 1
done
timeout -k 10 150 python -u bench.py --only count > gpurun_out/long/count.json 2> gpurun_out/long/count.err || exit 1

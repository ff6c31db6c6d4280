set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lstm_kernel.py tests/test_fused_policy.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lstm_test.log 2>&1 && \
timeout -k 10 120 python -u scripts/lstm_latency.py team > gpurun_out/lat_new.log 2>&1 && \
timeout -k 10 300 python -u bench.py --actor 0 > gpurun_out/bench.log 2>&1

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_tn.py tests/test_fused_policy.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fused_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --actor 0 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model 5v5 --steps 10 --warmup 3 --actor 0 > gpurun_out/bench_5v5.log 2>&1

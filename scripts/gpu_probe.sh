set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attn_kernels.py tests/test_fused_policy.py -x -q -k "attn or 5v5 or ln or pool or encoder" --timeout 200 --timeout-method thread > gpurun_out/attn_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model 5v5 --steps 10 --warmup 3 --actor 0 > gpurun_out/bench_5v5.log 2>&1

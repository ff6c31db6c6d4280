set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_policy.py tests/test_attn_kernels.py -x -v --timeout 120 --timeout-method thread > gpurun_out/fused_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --model 5v5 --steps 5 --warmup 2 --actor 0 > gpurun_out/bench_5v5.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model 5v5 --steps 3 --warmup 2 --actor 0 > $GRAFT_REPO_ROOT/gpurun_out/prof5.log 2>&1

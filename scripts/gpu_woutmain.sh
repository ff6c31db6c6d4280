# 5v5 tail A/B: dW_out on the main stream after the encoder backward vs both attention dW GEMMs on the side stream
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--model 5v5 --precision fp32 --steps 20 --warmup 5 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --actor 0 --e2e 0 --league-replay-extra 0 --e2e-5v5-extra 0"
DCA_WOUT_MAIN=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused_policy.py tests/test_fp32_kernels.py > gpurun_out/wm_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py $B > gpurun_out/wm0.log 2>&1 && \
DCA_WOUT_MAIN=1 timeout -k 10 200 python -u bench.py $B > gpurun_out/wm1.log 2>&1 && \
timeout -k 10 200 python -u bench.py $B > gpurun_out/wm0b.log 2>&1 && \
DCA_WOUT_MAIN=1 timeout -k 10 200 python -u bench.py $B > gpurun_out/wm1b.log 2>&1

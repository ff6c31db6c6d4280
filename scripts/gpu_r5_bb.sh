# round 5 (bb): 5v5 step with ∂W_qkv on a third stream (DCA_ATTN_WG3=1) vs both attention GEMMs on the side stream
set -o pipefail
mkdir -p gpurun_out
B="--steps 10 --warmup 3 --actor 0 --e2e 0 --bf16x3-extra 0 --model-5v5-extra 20 --model-5v5-exact-extra 10 --bptt350-extra 0 --big-batch-extra 0 --league-replay-extra 0 --e2e-5v5-extra 0"
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_exact_mode.py tests/test_fused_policy.py tests/test_attn_kernels.py > gpurun_out/r5_bb_tests.log 2>&1 && \
DCA_ATTN_WG3=1 timeout -k 10 300 python -u bench.py $B > gpurun_out/r5_bb_1.json 2> gpurun_out/r5_bb_1.err && \
DCA_ATTN_WG3=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/r5_bb_0.json 2> gpurun_out/r5_bb_0.err && \
DCA_ATTN_WG3=1 timeout -k 10 300 python -u bench.py $B > gpurun_out/r5_bb_1b.json 2> gpurun_out/r5_bb_1b.err
echo "rc=$?"
tail -2 gpurun_out/r5_bb_tests.log

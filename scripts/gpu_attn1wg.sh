# 5v5 attention-block forward: one workgroup per CU with prefetched weights vs two per CU
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--model 5v5 --precision fp32 --steps 10 --warmup 3 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --actor 0 --e2e 0 --league-replay-extra 0"
DCA_ATTN_FWD_1WG=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attn_kernels.py > gpurun_out/attn1_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py $B > gpurun_out/a2.log 2>&1 && \
DCA_ATTN_FWD_1WG=1 timeout -k 10 200 python -u bench.py $B > gpurun_out/a1.log 2>&1 && \
timeout -k 10 200 python -u bench.py $B > gpurun_out/a2b.log 2>&1 && \
DCA_ATTN_FWD_1WG=1 timeout -k 10 200 python -u bench.py $B > gpurun_out/a1b.log 2>&1

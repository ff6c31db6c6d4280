# tail ordering A/B: pre-RNN weight gradient on the main stream after the encoder backward vs on the side stream
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--steps 20 --warmup 5 --bf16x3-extra 1 --model-5v5-extra 1 --model-5v5-exact-extra 0 --bptt350-extra 0 --actor 0 --e2e 0 --league-replay-extra 0 --e2e-5v5-extra 0"
DCA_PRE_ON_MAIN=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_exact_mode.py tests/test_fused_policy.py > gpurun_out/pm_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py $B > gpurun_out/pm0.log 2>&1 && \
DCA_PRE_ON_MAIN=1 timeout -k 10 200 python -u bench.py $B > gpurun_out/pm1.log 2>&1 && \
timeout -k 10 200 python -u bench.py $B > gpurun_out/pm0b.log 2>&1 && \
DCA_PRE_ON_MAIN=1 timeout -k 10 200 python -u bench.py $B > gpurun_out/pm1b.log 2>&1

# fused dW_hh in the exact backward recurrence: numerics, headline A/B, kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--steps 20 --warmup 5 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --actor 0 --e2e 0 --league-replay-extra 0"
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_exact_mode.py tests/test_packing.py tests/test_fused_policy.py > gpurun_out/fdw_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py $B > gpurun_out/fdw_on.log 2> gpurun_out/fdw_on.err && \
DCA_FUSED_DW=0 timeout -k 10 200 python -u bench.py $B > gpurun_out/fdw_off.log 2> gpurun_out/fdw_off.err && \
timeout -k 10 200 python -u bench.py $B > gpurun_out/fdw_on2.log 2> gpurun_out/fdw_on2.err && \
bash scripts/prof_exact.sh proffdw

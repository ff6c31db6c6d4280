# exact learner step A/B: encoder backward in its 4-wave two-workgroups-per-CU form (DCA_ENC_BWD_X2=1, now the default) vs the 8-wave form
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--steps 20 --warmup 5 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --actor 0 --e2e 0 --league-replay-extra 0 --e2e-5v5-extra 0"
DCA_ENC_BWD_X2=0 timeout -k 10 200 python -u bench.py $B > gpurun_out/x0.log 2>&1 && \
DCA_ENC_BWD_X2=1 timeout -k 10 200 python -u bench.py $B > gpurun_out/x1.log 2>&1 && \
DCA_ENC_BWD_X2=0 timeout -k 10 200 python -u bench.py $B > gpurun_out/x0b.log 2>&1 && \
DCA_ENC_BWD_X2=1 timeout -k 10 200 python -u bench.py $B > gpurun_out/x1b.log 2>&1

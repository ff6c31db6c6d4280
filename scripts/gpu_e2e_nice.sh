# node loop: actor process CPU priority A/B (nice 0 vs 5 vs 10)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DCA_ACTOR_NICE=0 timeout -k 10 200 python -u scripts/e2e_ab.py 15 2048,14,bf16,1 > gpurun_out/e2e_nice0.log 2> gpurun_out/e2e_nice0.err && \
DCA_ACTOR_NICE=5 timeout -k 10 200 python -u scripts/e2e_ab.py 15 2048,14,bf16,1 > gpurun_out/e2e_nice5.log 2> gpurun_out/e2e_nice5.err && \
DCA_ACTOR_NICE=10 timeout -k 10 200 python -u scripts/e2e_ab.py 15 2048,14,bf16,1 2048,16,bf16,2 > gpurun_out/e2e_nice10.log 2> gpurun_out/e2e_nice10.err

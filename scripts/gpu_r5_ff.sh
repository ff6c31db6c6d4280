# round 5 (ff): node loop with the actor's step stream at default priority (0) vs high (-1, current)
set -o pipefail
mkdir -p gpurun_out
B="--steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 20 --league-replay-extra 0 --e2e-5v5-extra 0"
DCA_ACTOR_PRIORITY=0 timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_ff_0.json 2> gpurun_out/r5_ff_0.err && \
DCA_ACTOR_PRIORITY=-1 timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_ff_1.json 2> gpurun_out/r5_ff_1.err && \
DCA_ACTOR_PRIORITY=0 timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_ff_0b.json 2> gpurun_out/r5_ff_0b.err
echo "rc=$?"

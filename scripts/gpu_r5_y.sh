# round 5 (y): CU partition between the node loop's actor and learner (HSA_CU_MASK in the actor process only)
set -o pipefail
mkdir -p gpurun_out
B="--steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 15 --league-replay-extra 0 --e2e-5v5-extra 0"
DCA_ACTOR_CU_MASK="0:0-31" timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_y_a.json 2> gpurun_out/r5_y_a.err && \
DCA_ACTOR_CU_MASK="0:0-3,32-35,64-67,96-99,128-131,160-163,192-195,224-227" timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_y_b.json 2> gpurun_out/r5_y_b.err && \
DCA_ACTOR_CU_MASK="0:0-63" timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_y_c.json 2> gpurun_out/r5_y_c.err
echo "rc=$?"

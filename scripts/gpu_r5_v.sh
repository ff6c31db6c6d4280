# round 5 (v): GIL hand-off latency in the node loop's learner process and who holds it
set -o pipefail
mkdir -p gpurun_out
B="--steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 15 --league-replay-extra 0 --e2e-5v5-extra 0"
DCA_GIL_PROBE=1 DCA_STAGE_PROF=1 timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_v.json 2> gpurun_out/r5_v.err
echo "rc=$?"

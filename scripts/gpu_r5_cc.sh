# round 5 (cc): the node loop on smaller CPU shares — 4 and 8 actor threads instead of 14 (what 8 ranks on a
# 128-CPU node with a 16-CPU lease each, or tighter leases, would give the actor)
set -o pipefail
mkdir -p gpurun_out
B="--steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 15 --league-replay-extra 0 --e2e-5v5-extra 0"
timeout -k 10 240 python -u bench.py $B --e2e-threads 4 > gpurun_out/r5_cc_4.json 2> gpurun_out/r5_cc_4.err && \
timeout -k 10 240 python -u bench.py $B --e2e-threads 8 > gpurun_out/r5_cc_8.json 2> gpurun_out/r5_cc_8.err
echo "rc=$?"

# round 5 (q): node loop with the stager's time split (slot wait / field copies / ring releases)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 20 --league-replay-extra 0 --e2e-5v5-extra 0 > gpurun_out/r5_e2e_q.json 2> gpurun_out/r5_e2e_q.err
echo "rc=$?"

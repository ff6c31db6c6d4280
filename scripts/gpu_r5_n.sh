# round 5 (n): node loop with zero-copy consumption wired into the stager pipeline; config 5 with and without the
# replay prefill (isolates the config-5 stall)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 20 --league-replay-extra 15 --e2e-5v5-extra 0 > gpurun_out/r5_e2e_n.json 2> gpurun_out/r5_e2e_n.err && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 0 --league-replay-extra 15 --league-replay-prefill 0 --e2e-5v5-extra 0 > gpurun_out/r5_e2e_n2.json 2> gpurun_out/r5_e2e_n2.err
echo "rc=$?"

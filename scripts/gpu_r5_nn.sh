# round 5 (nn): short bench sanity after the bench-wide hand-off deadline change
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 10 --league-replay-extra 0 --e2e-5v5-extra 0 > gpurun_out/r5_nn.json 2> gpurun_out/r5_nn.err
echo "rc=$?"

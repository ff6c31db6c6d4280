# round 5 (i): pointer-head diagnostic of the exact 5v5 step; node loop with the actor's in-place ring publish
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/diag_5v5_head.py 1400 > gpurun_out/r5_diag_5v5_head.txt 2>&1
echo "diag rc=$?"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 20 --league-replay-extra 15 --e2e-5v5-extra 15 > gpurun_out/r5_e2e_sink.json 2> gpurun_out/r5_e2e_sink.err
echo "e2e rc=$?"

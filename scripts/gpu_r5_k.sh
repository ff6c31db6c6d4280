set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/diag_5v5_head.py 1400 > gpurun_out/r5_diag_5v5_head4.txt 2>&1
echo "diag rc=$?"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 1 --e2e 20 --league-replay-extra 0 --e2e-5v5-extra 0 > gpurun_out/r5_e2e_stage.json 2> gpurun_out/r5_e2e_stage.err
echo "e2e rc=$?"
DCA_TEAM_HALF=1 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 20 --league-replay-extra 0 --e2e-5v5-extra 0 > gpurun_out/r5_e2e_half.json 2> gpurun_out/r5_e2e_half.err
echo "e2e half rc=$?"

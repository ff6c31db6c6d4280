# round 5 (gg): node loop with 2048 / 4096 / 6144 actor games (default 3072); /dev/shm size of the box
set -o pipefail
mkdir -p gpurun_out
df -h /dev/shm > gpurun_out/r5_gg_shm.txt
B="--steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 20 --league-replay-extra 0 --e2e-5v5-extra 0"
timeout -k 10 240 python -u bench.py $B --e2e-games 4096 > gpurun_out/r5_gg_4096.json 2> gpurun_out/r5_gg_4096.err && \
timeout -k 10 240 python -u bench.py $B --e2e-games 6144 > gpurun_out/r5_gg_6144.json 2> gpurun_out/r5_gg_6144.err && \
timeout -k 10 240 python -u bench.py $B --e2e-games 2048 > gpurun_out/r5_gg_2048.json 2> gpurun_out/r5_gg_2048.err
echo "rc=$?"

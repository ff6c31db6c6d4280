# round 5 (jj): config-5 loop twice more after the fused-expand change (r5_ii_a saw one 11 s device stall in it)
set -o pipefail
mkdir -p gpurun_out
{ rocm-smi --showmeminfo vram 2>&1 | grep -i "used" ; } > gpurun_out/r5_jj_mem.txt || true
B="--steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 0 --league-replay-extra 15 --e2e-5v5-extra 0"
timeout -k 10 300 python -u bench.py $B > gpurun_out/r5_jj_a.json 2> gpurun_out/r5_jj_a.err && \
timeout -k 10 300 python -u bench.py $B > gpurun_out/r5_jj_b.json 2> gpurun_out/r5_jj_b.err
echo "rc=$?"

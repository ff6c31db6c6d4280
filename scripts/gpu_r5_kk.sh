# round 5 (kk): config-5 stalls — same box, the fused expand / normalisation kernels off (torch path) vs on
set -o pipefail
mkdir -p gpurun_out
{ rocm-smi --showmeminfo vram 2>&1 | grep -i "used" ; rocm-smi --showpids 2>&1 | tail -8 ; } > gpurun_out/r5_kk_mem.txt || true
B="--steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 0 --league-replay-extra 15 --e2e-5v5-extra 0"
DCA_DIAG_TORCH_EXPAND=1 timeout -k 10 300 python -u bench.py $B > gpurun_out/r5_kk_t.json 2> gpurun_out/r5_kk_t.err && \
timeout -k 10 300 python -u bench.py $B > gpurun_out/r5_kk_k.json 2> gpurun_out/r5_kk_k.err
echo "rc=$?"

# round 5 (mm): fused ingest kernels A/B on one box — config 5 first (fresh process), then e2e K/T/K/T
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_returns_scan.py > gpurun_out/r5_mm_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 0 --league-replay-extra 15 --e2e-5v5-extra 0 > gpurun_out/r5_mm_l.json 2> gpurun_out/r5_mm_l.err && \
B="--steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 20 --league-replay-extra 0 --e2e-5v5-extra 0" && \
timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_mm_k1.json 2> gpurun_out/r5_mm_k1.err && \
DCA_AB_TORCH_EXPAND=1 timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_mm_t1.json 2> gpurun_out/r5_mm_t1.err && \
timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_mm_k2.json 2> gpurun_out/r5_mm_k2.err && \
DCA_AB_TORCH_EXPAND=1 timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_mm_t2.json 2> gpurun_out/r5_mm_t2.err
echo "rc=$?"
tail -1 gpurun_out/r5_mm_tests.log

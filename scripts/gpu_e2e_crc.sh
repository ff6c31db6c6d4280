# node loop after the CRC-32C combine fix: bench e2e field + 1 vs 2 actor processes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --actor 0 --league-replay-extra 0 > gpurun_out/e2e_crc_bench.log 2> gpurun_out/e2e_crc_bench.err && \
timeout -k 10 300 python -u scripts/e2e_ab.py 15 2048,14,bf16,1 2048,16,bf16,2 > gpurun_out/e2e_ab7.log 2> gpurun_out/e2e_ab7.err

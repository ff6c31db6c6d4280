# round 5 (s): node loop with the stager's native field packing (pack_rows), stage sections profiled
set -o pipefail
mkdir -p gpurun_out
B="--steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 20 --league-replay-extra 0 --e2e-5v5-extra 0"
DCA_STAGE_PROF=1 timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_s_t1.json 2> gpurun_out/r5_s_t1.err && \
DCA_STAGE_PROF=1 DCA_DECODE_THREADS=2 timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_s_t2.json 2> gpurun_out/r5_s_t2.err
echo "rc=$?"

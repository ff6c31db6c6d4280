# round 5 (r): stager GIL contention A/B — zero-copy decode threads 1 vs 3, GIL switch interval 5 ms vs 0.5 ms
set -o pipefail
mkdir -p gpurun_out
B="--steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 15 --league-replay-extra 0 --e2e-5v5-extra 0"
DCA_STAGE_PROF=1 DCA_DECODE_THREADS=1 timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_r_t1.json 2> gpurun_out/r5_r_t1.err && \
DCA_STAGE_PROF=1 DCA_DECODE_THREADS=3 timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_r_t3.json 2> gpurun_out/r5_r_t3.err && \
DCA_DECODE_THREADS=1 DCA_SWITCH_INTERVAL=0.0005 DCA_STAGE_PROF=1 timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_r_t1s.json 2> gpurun_out/r5_r_t1s.err
echo "rc=$?"

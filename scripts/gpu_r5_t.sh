# round 5 (t): what holds the learner's GIL while the stager waits — baseline / 0.2 ms switch interval / no files
set -o pipefail
mkdir -p gpurun_out
B="--steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 15 --league-replay-extra 0 --e2e-5v5-extra 0"
DCA_STAGE_PROF=1 DCA_SWITCH_INTERVAL=0.0002 timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_t_si.json 2> gpurun_out/r5_t_si.err && \
DCA_STAGE_PROF=1 DCA_DIAG_SKIP_FILES=1 timeout -k 10 240 python -u bench.py $B > gpurun_out/r5_t_nf.json 2> gpurun_out/r5_t_nf.err
echo "rc=$?"

# round 5 (x): node loops with the default 2 s recurrence hand-off timeout (no DCA_TEAM_PATIENT) now that the
# config-5 stall's cause (ring claims leaked by the host ingest path) is fixed — e2e, config 5, config 4
set -o pipefail
mkdir -p gpurun_out
B="--steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 20 --league-replay-extra 20 --e2e-5v5-extra 20"
DCA_TEAM_PATIENT=0 timeout -k 10 400 python -u bench.py $B > gpurun_out/r5_x.json 2> gpurun_out/r5_x.err
echo "rc=$?"

# round 6 (n): hardware queues of the node loop's ACTOR process only (DCA_E2E_ACTOR_HW_QUEUES → its GPU_MAX_HW_QUEUES):
# fewer queues from the other process beside the learner's persistent recurrence; default (4) first and last
set -o pipefail
mkdir -p gpurun_out
E="--bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --league-replay-extra 0 --e2e-5v5-extra 0"
run() {
  DCA_E2E_ACTOR_HW_QUEUES=$2 timeout -k 10 300 python -u bench.py $E > gpurun_out/r6n_bench_$1.json 2> gpurun_out/r6n_bench_$1.err
}
run q4 4 && run q1 1 && run q2 2 && run q4b 4 && run q1b 1 || exit $?
echo done

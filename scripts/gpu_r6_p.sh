# round 6 (p): the node loop's actor launch shape — 1 / 2 (default) / 4 software-pipelined game groups in the actor
# process (DCA_E2E_ACTOR_GROUPS): does the learner's in-loop slowdown follow the actor's launch granularity?
set -o pipefail
mkdir -p gpurun_out
E="--bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --league-replay-extra 0 --e2e-5v5-extra 0 --e2e-extra 0"
run() {
  DCA_E2E_ACTOR_GROUPS=$2 timeout -k 10 300 python -u bench.py $E > gpurun_out/r6p_bench_$1.json 2> gpurun_out/r6p_bench_$1.err
}
run g2 2 && run g1 1 && run g4 4 && run g2b 2 && run g4b 4 || exit $?
echo done

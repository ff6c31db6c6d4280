# round 6 (q): the node loop's learner step alone (in-step V-trace) next to the headline step, and the e2e loop on
# the same box — how much of the in-loop 6.9 ms is V-trace work and how much is interference
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 \
  --big-batch-extra 0 --actor 0 --league-replay-extra 0 --e2e-5v5-extra 0 --e2e-extra 0 > gpurun_out/r6q_bench.json 2> gpurun_out/r6q_bench.err || exit $?
echo done

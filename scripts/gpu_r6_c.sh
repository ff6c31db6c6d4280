# round 6 (c): policy_old diagnostic, node-loop A/B (actor precision, old_logp, actor copies in/out of the graph),
# the 5v5 node loop, and the exact recurrence's per-phase trace
set -o pipefail
mkdir -p gpurun_out
E2E="--steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --league-replay-extra 0 --e2e-5v5-extra 0 --e2e-extra 0 --e2e 15"
timeout -k 10 400 python -u scripts/offpolicy_diag.py > gpurun_out/r6c_offdiag.jsonl 2> gpurun_out/r6c_offdiag.err && \
timeout -k 10 300 python -u bench.py $E2E > gpurun_out/r6c_e2e_fp32_learner.json 2> gpurun_out/r6c_e2e_fp32_learner.err && \
timeout -k 10 300 python -u bench.py $E2E --e2e-old-logp actor > gpurun_out/r6c_e2e_fp32_actor.json 2> gpurun_out/r6c_e2e_fp32_actor.err && \
DCA_ACTOR_GRAPH_COPIES=1 timeout -k 10 300 python -u bench.py $E2E > gpurun_out/r6c_e2e_fp32_learner_gcopy.json 2> gpurun_out/r6c_e2e_fp32_learner_gcopy.err && \
timeout -k 10 300 python -u bench.py $E2E --e2e-actor-precision bf16 --e2e-old-logp actor > gpurun_out/r6c_e2e_bf16_actor.json 2> gpurun_out/r6c_e2e_bf16_actor.err && \
timeout -k 10 120 python -u scripts/lstm_team_trace.py f32 > gpurun_out/r6c_trace_fwd.jsonl 2>&1 && \
timeout -k 10 120 python -u scripts/lstm_team_trace.py f32 bwd > gpurun_out/r6c_trace_bwd.jsonl 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --league-replay-extra 0 --e2e 0 --e2e-extra 0 --e2e-5v5-extra 15 > gpurun_out/r6c_e2e5v5.json 2> gpurun_out/r6c_e2e5v5.err
echo "exit $?"

# round 6 (b): GPU suite minus the 30 s learning test, then that test's loop as an A/B of the learner-side policy_old
# (old_logp learner vs actor, same seed), then the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  --deselect tests/test_learning.py::test_short_training_beats_the_untrained_policy_vs_default_bot \
  > gpurun_out/r6b_gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u scripts/learning_curve.py --budget 40 --eval-every 20 --eval-games 128 --games 1024 \
  --threads 12 --snapshot-lags '' --old-logp learner --out gpurun_out/r6b_curve_learner.jsonl > gpurun_out/r6b_curve_learner.log 2>&1 && \
timeout -k 10 300 python -u scripts/learning_curve.py --budget 40 --eval-every 20 --eval-games 128 --games 1024 \
  --threads 12 --snapshot-lags '' --old-logp actor --out gpurun_out/r6b_curve_actor.jsonl > gpurun_out/r6b_curve_actor.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6b_smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6b_bench.json 2> gpurun_out/r6b_bench.err
echo "exit $?"

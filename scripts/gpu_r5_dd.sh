# round 5 (dd): node loop + ring GPU tests after the monotonic-token / claim-abandonment ring change
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_vec_actor.py tests/test_learner_async.py > gpurun_out/r5_dd_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 20 --league-replay-extra 15 --e2e-5v5-extra 0 > gpurun_out/r5_dd.json 2> gpurun_out/r5_dd.err
echo "rc=$?"
tail -1 gpurun_out/r5_dd_tests.log

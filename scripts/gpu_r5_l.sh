# round 5 (l): exact tests after the heads_loss p = e/s change, the learner-async tests, the node loop with 3 decode
# threads on the zero-copy ring path
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_exact_mode.py tests/test_learner_async.py tests/test_determinism.py -m gpu > gpurun_out/r5_l_tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 20 --league-replay-extra 15 --e2e-5v5-extra 0 > gpurun_out/r5_e2e_mt.json 2> gpurun_out/r5_e2e_mt.err
echo "e2e rc=$?"

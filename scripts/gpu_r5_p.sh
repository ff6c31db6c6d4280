# round 5 (p): async host snapshot of the per-iteration device values (no finalize syncs) — optimizer GPU tests +
# node loop with the stage-wait split
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_learner_async.py tests/test_replay.py tests/test_returns_scan.py > gpurun_out/r5_p_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 20 --league-replay-extra 0 --e2e-5v5-extra 0 > gpurun_out/r5_e2e_p.json 2> gpurun_out/r5_e2e_p.err
echo "rc=$?"
tail -3 gpurun_out/r5_p_tests.log

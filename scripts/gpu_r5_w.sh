# round 5 (w): returns-scan metadata uploaded non-blocking (no GIL-held stream wait in the look-ahead ingest)
set -o pipefail
mkdir -p gpurun_out
B="--steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 20 --league-replay-extra 15 --e2e-5v5-extra 0"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_returns_scan.py tests/test_learner_async.py > gpurun_out/r5_w_tests.log 2>&1 && \
DCA_GIL_PROBE=1 DCA_STAGE_PROF=1 timeout -k 10 300 python -u bench.py $B > gpurun_out/r5_w.json 2> gpurun_out/r5_w.err
echo "rc=$?"
tail -2 gpurun_out/r5_w_tests.log

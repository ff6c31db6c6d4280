# round 5 (ii): fused look-ahead expand (ingest_scatter) + advantage normalisation — tests and node loop
set -o pipefail
mkdir -p gpurun_out
B="--steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 20 --league-replay-extra 15 --e2e-5v5-extra 15"
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_returns_scan.py tests/test_learner_async.py tests/test_learning.py tests/test_replay.py tests/test_packing.py > gpurun_out/r5_ii_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py $B > gpurun_out/r5_ii_a.json 2> gpurun_out/r5_ii_a.err && \
timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 20 --league-replay-extra 0 --e2e-5v5-extra 0 > gpurun_out/r5_ii_b.json 2> gpurun_out/r5_ii_b.err
echo "rc=$?"
tail -1 gpurun_out/r5_ii_tests.log

# round 6 (d): GPU tests of the in-step V-trace / split-K fold / pipeline, then 1v1 curves at the bench's node-loop
# shape (3072 games: weight age ≈ 12-22) — in-step V-trace vs the round-5 GAE — then the full bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest \
  tests/test_learner_async.py \
  tests/test_dp_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r6d_gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u scripts/learning_curve.py --budget 120 --eval-every 40 --eval-games 128 --games 3072 \
  --threads 12 --snapshot-lags '' --advantages vtrace-step --out gpurun_out/r6d_curve_vtrace3072.jsonl > gpurun_out/r6d_curve_vtrace3072.log 2>&1 && \
timeout -k 10 400 python -u scripts/learning_curve.py --budget 120 --eval-every 40 --eval-games 128 --games 3072 \
  --threads 12 --snapshot-lags '' --advantages gae --out gpurun_out/r6d_curve_gae3072.jsonl > gpurun_out/r6d_curve_gae3072.log 2>&1 && \
timeout -k 10 700 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6d_bench.json 2> gpurun_out/r6d_bench.err
echo "exit $?"

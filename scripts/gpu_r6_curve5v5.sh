# round 6: 5v5 learning curve (BASELINE config 4: entity attention, fp32-exact learner with in-step V-trace, 5v5
# self-play actors on the IEEE-fp32 policy step) — default-bot win rate AND head-to-head games against the weights
# of 2 / 5 / 10 minutes of training earlier (the default-bot rate saturates within 90 s); resumable via --log-dir
set -o pipefail
mkdir -p gpurun_out
# (first: the split-count change in the TN GEMM plan — exact-mode parity and the standalone kernel timings)
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_exact_mode.py \
  > gpurun_out/r6g_exact_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/exact_kernels_bench.py 10 > gpurun_out/r6g_kernels.txt 2>&1 || exit $?
timeout -k 10 1000 python -u scripts/learning_curve.py --model 5v5 --mode 5v5 --eval-precision fp32 --actor-precision fp32 \
  --games 400 --budget 720 --eval-every 90 --eval-games 128 --snapshot-lags 120,300,600 --snapshot-games 64 \
  --log-dir /tmp/r6_curve5v5_ckpt --out gpurun_out/r6_curve_5v5.jsonl > gpurun_out/r6_curve_5v5.log 2>&1
echo "curve rc=$?"

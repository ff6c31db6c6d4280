# round 6: 5v5 learning curve (BASELINE config 4: entity attention, fp32-exact learner with in-step V-trace, 5v5
# self-play actors on the IEEE-fp32 policy step) — default-bot win rate AND head-to-head games against the weights
# of 2 / 5 / 10 minutes of training earlier (the default-bot rate saturates within 90 s); resumable via --log-dir
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1150 python -u scripts/learning_curve.py --model 5v5 --mode 5v5 --eval-precision fp32 --actor-precision fp32 \
  --games 400 --budget 720 --eval-every 90 --eval-games 128 --snapshot-lags 120,300,600 --snapshot-games 64 \
  --log-dir gpurun_out/r6_curve5v5_ckpt --out gpurun_out/r6_curve_5v5.jsonl > gpurun_out/r6_curve_5v5.log 2>&1
echo "curve rc=$?"

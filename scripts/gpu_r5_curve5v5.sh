# round 5: 5v5 learning curve (BASELINE config 4 policy, fp32-exact learner, 5v5 self-play actors) against the
# scripted default bot (five controlled heroes), 12 min of training
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1120 python -u scripts/learning_curve.py --model 5v5 --mode 5v5 --eval-precision bf16 --games 400 \
  --budget 720 --eval-every 90 --eval-games 128 --out gpurun_out/r5_curve_5v5.jsonl > gpurun_out/r5_curve_5v5.log 2>&1
echo "curve rc=$?"

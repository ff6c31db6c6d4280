# round 5: 1v1 learning curves at two more seeds (8 min of training each) — is the win-rate gain reproducible?
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 560 python -u scripts/learning_curve.py --budget 480 --eval-every 60 --eval-games 256 --seed 11 \
  --out gpurun_out/r5_curve_1v1_seed11.jsonl > gpurun_out/r5_curve_1v1_seed11.log 2>&1 && \
timeout -k 10 560 python -u scripts/learning_curve.py --budget 480 --eval-every 60 --eval-games 256 --seed 23 \
  --out gpurun_out/r5_curve_1v1_seed23.jsonl > gpurun_out/r5_curve_1v1_seed23.log 2>&1
echo "rc=$?"

# round 6: BASELINE config 5 as a curve again, the learner sampling the replay's 4 096 newest sequences (≈4 s of
# experience at the loop's rate) instead of the whole 100 GB buffer (profiles/r6_curve_league.jsonl: uniform sampling
# over all experience so far learns the default-bot game slowly)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/learning_curve.py --budget 600 --eval-every 75 --eval-games 256 \
  --league pfsp --latest-weights-prob 0.8 --actor-precision fp8 --replay-gb 100 --replay-recent 4096 \
  --snapshot-lags 120,300,600 --snapshot-games 64 --league-matrix 4 --out gpurun_out/r6_curve_league_recent.jsonl \
  > gpurun_out/r6_curve_league_recent.log 2>&1
echo "curve rc=$?"

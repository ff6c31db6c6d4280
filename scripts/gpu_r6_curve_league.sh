# round 6: BASELINE config 5 as a learning curve after the stall fix (default 2 s hand-off deadline) — PFSP self-play
# league, fp8 actor policy step, every minibatch from a 100 GB on-HBM replay with the in-step V-trace (advantages
# recomputed at every sampling from the weights being trained); default-bot win rate (fp32 actor), head-to-head vs
# the weights of 2 / 5 / 10 minutes earlier, the league's score against its pool, and a 4-snapshot win-rate matrix
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1150 python -u scripts/learning_curve.py --budget 600 --eval-every 75 --eval-games 256 \
  --league pfsp --latest-weights-prob 0.8 --actor-precision fp8 --replay-gb 100 --snapshot-lags 120,300,600 \
  --snapshot-games 64 --league-matrix 4 --out gpurun_out/r6_curve_league.jsonl > gpurun_out/r6_curve_league.log 2>&1
echo "curve rc=$?"

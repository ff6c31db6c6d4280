# round 6 (o): the final stack as the node loop runs it — GPU featurization (raw unit records), the IEEE-fp32 actor,
# in-step V-trace, actors 16 versions behind (the bench's weight age) — a 10-minute 1v1 curve with snapshot evaluation
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u scripts/learning_curve.py --budget 600 --eval-every 100 --eval-games 256 --games 1024 \
  --threads 12 --actor-precision fp32 --weight-lag 16 --advantages vtrace-step --snapshot-lags 200,400 \
  --snapshot-games 64 --out gpurun_out/r6_curve_1v1_final.jsonl > gpurun_out/r6_curve_1v1_final.log 2>&1
echo "curve rc=$?"

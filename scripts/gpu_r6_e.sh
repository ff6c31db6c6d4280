# round 6 (e): full bench with the split-K fold back off (default); then 1v1 learning curves at forced staleness
# (actors 16 versions behind: the node loop's weight age) — in-step V-trace vs the round-5 GAE on actor values
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6e_bench.json 2> gpurun_out/r6e_bench.err && \
timeout -k 10 400 python -u scripts/learning_curve.py --budget 150 --eval-every 50 --eval-games 128 --games 1024 \
  --threads 12 --snapshot-lags '' --weight-lag 16 --advantages vtrace-step --out gpurun_out/r6e_curve_lag16_vtrace.jsonl > gpurun_out/r6e_curve_lag16_vtrace.log 2>&1 && \
timeout -k 10 400 python -u scripts/learning_curve.py --budget 150 --eval-every 50 --eval-games 128 --games 1024 \
  --threads 12 --snapshot-lags '' --weight-lag 16 --advantages gae --out gpurun_out/r6e_curve_lag16_gae.jsonl > gpurun_out/r6e_curve_lag16_gae.log 2>&1
echo "exit $?"

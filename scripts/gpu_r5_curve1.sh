# round 5: 1v1 learning curve, part 1 of 2 (14 min of training; checkpoint + curve state under gpurun_out/ so the
# second call resumes it — scripts/learning_curve.py --log-dir)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1120 python -u scripts/learning_curve.py --budget 840 --eval-every 60 --eval-games 256 \
  --log-dir gpurun_out/r5_curve1v1_ckpt --out gpurun_out/r5_curve_1v1.jsonl > gpurun_out/r5_curve_1v1.log 2>&1
echo "curve rc=$?"
# only what the resume reads travels back (gpurun merges gpurun_out/ only below 64 MiB): the newest checkpoint pair
# and curve_state.json — the per-iteration metrics.jsonl (≈40 MB over 14 min) and event files stay on the box
rm -f gpurun_out/r5_curve1v1_ckpt/*.tfevents* gpurun_out/r5_curve1v1_ckpt/events.* gpurun_out/r5_curve1v1_ckpt/metrics.jsonl
ls -la gpurun_out/r5_curve1v1_ckpt
du -sh gpurun_out
if [ "$(du -sm gpurun_out | cut -f1)" -gt 60 ]; then mv gpurun_out/r5_curve1v1_ckpt /tmp/ && echo "checkpoint too large to return"; fi

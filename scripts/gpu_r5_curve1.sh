# round 5: 1v1 learning curve, part 1 of 2 (14 min of training; checkpoint + curve state under gpurun_out/ so the
# second call resumes it — scripts/learning_curve.py --log-dir)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1120 python -u scripts/learning_curve.py --budget 840 --eval-every 60 --eval-games 256 \
  --log-dir gpurun_out/r5_curve1v1_ckpt --out gpurun_out/r5_curve_1v1.jsonl > gpurun_out/r5_curve_1v1.log 2>&1
echo "curve rc=$?"
rm -f gpurun_out/r5_curve1v1_ckpt/*.tfevents* gpurun_out/r5_curve1v1_ckpt/events.* 2>/dev/null
du -sh gpurun_out/r5_curve1v1_ckpt

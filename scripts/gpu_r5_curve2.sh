# round 5: 1v1 learning curve, part 2 of 2 — resumes runs/r5_curve1v1_ckpt (part 1's checkpoint, copied into the
# tree) to 28 min of training in total, saves the final weights, then the actor-precision check at those weights
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u scripts/learning_curve.py --budget 1680 --eval-every 60 --eval-games 256 \
  --log-dir runs/r5_curve1v1_ckpt --out gpurun_out/r5_curve_1v1_part2.jsonl \
  --save-model gpurun_out/r5_curve_1v1_model.pt > gpurun_out/r5_curve_1v1_part2.log 2>&1
echo "curve rc=$?"
timeout -k 10 300 python -u scripts/actor_precision_check.py --model gpurun_out/r5_curve_1v1_model.pt \
  --label trained-28min --out gpurun_out/r5_actor_precision_trained.jsonl > gpurun_out/r5_actor_precision_trained.log 2>&1
echo "precision check rc=$?"

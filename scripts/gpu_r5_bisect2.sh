# round 5: the league case of the stall bisection again with the actor's step streams at the default priority
# (2 s hand-off deadline), then the full config-5 combination
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  timeout -k 10 400 python -u scripts/learning_curve.py --budget 120 --eval-every 60 --eval-games 64 "$@" \
    --out gpurun_out/r5_bisect2_$tag.jsonl > gpurun_out/r5_bisect2_$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc" | tee -a gpurun_out/r5_bisect2_rc.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
rm -f gpurun_out/r5_bisect2_rc.txt
run league_bf16 --league pfsp --actor-precision bf16 && \
run config5 --league pfsp --actor-precision fp8 --replay-gb 100
echo done

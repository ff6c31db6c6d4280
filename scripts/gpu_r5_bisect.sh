# round 5: bisect the config-5 stalls at the default 2 s hand-off deadline — which of league / fp8 actor / replay
# triggers them? Short curves (120 s of training). A soft hand-off timeout ends a run with status 1 (the kernel exits
# cleanly through its error flag); any other failure status stops the script.
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  timeout -k 10 400 python -u scripts/learning_curve.py --budget 120 --eval-every 60 --eval-games 64 "$@" \
    --out gpurun_out/r5_bisect_$tag.jsonl > gpurun_out/r5_bisect_$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc" | tee -a gpurun_out/r5_bisect_rc.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
rm -f gpurun_out/r5_bisect_rc.txt
run league_bf16 --league pfsp --actor-precision bf16 && \
run fp8_only --actor-precision fp8 && \
run replay_only --actor-precision bf16 --replay-gb 100
echo done

# round 5 (d): full default bench, actor precision check (random init), actor + compat-step kernel summaries
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u bench.py > gpurun_out/r5_bench_full.json 2> gpurun_out/r5_bench_full.err || exit $?
timeout -k 10 300 python -u scripts/actor_precision_check.py --label random-init --out gpurun_out/r5_actor_precision.jsonl > gpurun_out/r5_actor_precision.log 2>&1 || exit $?
for P in fp32 bf16 fp8; do
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profa_$P -o run -- python3 $R/scripts/actor_bench.py 2048 $P > $R/gpurun_out/profa_$P.log 2>&1 || exit $?
  cd $R && python scripts/prof_summary.py gpurun_out/profa_$P/run_results.db --steps 111 > gpurun_out/r5_actor_${P}_summary.md && rm -rf gpurun_out/profa_$P || exit $?
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profc -o run -- python3 $R/bench.py --model compat --algo vpg --precision fp32-exact --steps 5 --warmup 3 --actor 0 --e2e 0 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --league-replay-extra 0 --e2e-5v5-extra 0 > $R/gpurun_out/r5_compat_prof.log 2>&1 || exit $?
cd $R && python scripts/prof_summary.py gpurun_out/profc/run_results.db --steps 9 > gpurun_out/r5_compat_summary.md && python scripts/step_timeline.py gpurun_out/profc/run_results.db > gpurun_out/r5_compat_timeline.txt && rm -rf gpurun_out/profc

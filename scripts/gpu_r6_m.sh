# round 6 (m): kernel summaries + one-step timelines of the 5v5 fp32-exact step (balanced weight-gradient streams, the
# TN GEMM plan fix) and the 1v1 headline step, then the config-5 curve on the replay's newest sequences
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
X="--steps 5 --warmup 3 --actor 0 --e2e 0 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --league-replay-extra 0 --e2e-5v5-extra 0"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof5x -o run -- python3 $R/bench.py --model 5v5 --precision fp32-exact $X > $R/gpurun_out/prof5x.log 2>&1 || exit $?
cd $R && python scripts/prof_summary.py gpurun_out/prof5x/run_results.db --steps 9 > gpurun_out/r6_5v5_exact_summary.md && python scripts/step_timeline.py gpurun_out/prof5x/run_results.db > gpurun_out/r6_5v5_exact_timeline.txt && rm -rf gpurun_out/prof5x || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof1 -o run -- python3 $R/bench.py $X > $R/gpurun_out/prof1.log 2>&1 || exit $?
cd $R && python scripts/prof_summary.py gpurun_out/prof1/run_results.db --steps 9 > gpurun_out/r6_final_exact_summary.md && python scripts/step_timeline.py gpurun_out/prof1/run_results.db > gpurun_out/r6_final_exact_timeline.txt && rm -rf gpurun_out/prof1 || exit $?
bash scripts/gpu_r6_curve_league_recent.sh

# round 6 (zz): kernel summary + one-step timeline of the 1v1 headline step on the final tree
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
X="--steps 5 --warmup 3 --actor 0 --e2e 0 --bf16x3-extra 0 --vtrace-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --league-replay-extra 0 --e2e-5v5-extra 0"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof1 -o run -- python3 $R/bench.py $X > $R/gpurun_out/prof1.log 2>&1 || exit $?
cd $R && python scripts/prof_summary.py gpurun_out/prof1/run_results.db --steps 9 > gpurun_out/r6_final2_exact_summary.md && python scripts/step_timeline.py gpurun_out/prof1/run_results.db > gpurun_out/r6_final2_exact_timeline.txt && rm -rf gpurun_out/prof1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --actor 0 --e2e 0 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --league-replay-extra 0 --e2e-5v5-extra 0 > gpurun_out/r6zz_learner.json 2> gpurun_out/r6zz_learner.err || exit $?
echo done

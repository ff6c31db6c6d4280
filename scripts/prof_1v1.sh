# rocprofv3 kernel summary + one-step timeline of the fp32 1v1 learner step (lstm512, B=8, S=1400), on the box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --precision fp32 --steps 5 --warmup 3 --actor 0 --e2e 0 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --league-replay-extra 0 --e2e-5v5-extra 0 > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1 && \
 cd $GRAFT_REPO_ROOT && python scripts/prof_summary.py gpurun_out/prof1/run_results.db --steps 9 > gpurun_out/prof1_summary.md && \
 python scripts/step_timeline.py gpurun_out/prof1/run_results.db > gpurun_out/prof1_timeline.txt && rm -rf gpurun_out/prof1

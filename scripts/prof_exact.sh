# rocprofv3 kernel summary + one-step timeline of the IEEE-fp32 (fp32-exact) 1v1 learner step (lstm512, B=8, S=1400)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-profx}
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --precision fp32-exact --steps 5 --warmup 3 --actor 0 --e2e 0 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --league-replay-extra 0 --e2e-5v5-extra 0 > $GRAFT_REPO_ROOT/gpurun_out/$TAG.log 2>&1 && \
 cd $GRAFT_REPO_ROOT && python scripts/prof_summary.py gpurun_out/$TAG/run_results.db --steps 9 > gpurun_out/${TAG}_summary.md && \
 python scripts/step_timeline.py gpurun_out/$TAG/run_results.db > gpurun_out/${TAG}_timeline.txt && rm -rf gpurun_out/$TAG

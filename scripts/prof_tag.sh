# rocprofv3 kernel summary + one-step timeline of the fp32 1v1 learner step under the caller's env (A/B of kernel
# variants): bash scripts/prof_tag.sh TAG  → gpurun_out/prof_TAG_summary.md, gpurun_out/prof_TAG_timeline.txt
set -o pipefail
TAG=$1
mkdir -p $GRAFT_REPO_ROOT/gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --precision fp32 --steps 5 --warmup 3 --actor 0 --e2e 0 --e2e-5v5-extra 0 --bf16x3-extra 0 --model-5v5-extra 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1 && \
 cd $GRAFT_REPO_ROOT && python scripts/prof_summary.py gpurun_out/prof_$TAG/run_results.db --steps 9 > gpurun_out/prof_${TAG}_summary.md && \
 python scripts/step_timeline.py gpurun_out/prof_$TAG/run_results.db > gpurun_out/prof_${TAG}_timeline.txt && rm -rf gpurun_out/prof_$TAG

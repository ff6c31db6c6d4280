# rocprofv3 kernel summaries of the batched GPU actor step, bf16 and fp8 (4096 player slots)
set -o pipefail
mkdir -p $GRAFT_REPO_ROOT/gpurun_out
export TMPDIR=/tmp
for P in bf16 fp8; do
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/profa_$P -o run -- python3 $GRAFT_REPO_ROOT/scripts/actor_bench.py 2048 $P > $GRAFT_REPO_ROOT/gpurun_out/profa_$P.log 2>&1 || exit $?
  cd $GRAFT_REPO_ROOT && python scripts/prof_summary.py gpurun_out/profa_$P/run_results.db --steps 111 > gpurun_out/profa_${P}_summary.md && rm -rf gpurun_out/profa_$P || exit $?
done

# exact learner step vs the split-K GEMM workgroup target (weight-gradient GEMMs in the tail)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--steps 20 --warmup 5 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --actor 0 --e2e 0 --league-replay-extra 0 --e2e-5v5-extra 0"
for t in 512 256 768 1024 512 256 768 1024; do
  DCA_GEMM_TN_TARGET=$t timeout -k 10 200 python -u bench.py $B > gpurun_out/gt_$t.log 2>&1 || exit $?
  echo "target $t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gt_$t.log | head -1)" >> gpurun_out/gt_summary.txt
done

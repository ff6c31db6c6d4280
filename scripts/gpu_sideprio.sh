# exact learner step (and 5v5 step) with the side stream at default vs high priority, graph and eager replay
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/sp_summary.txt
B="--steps 20 --warmup 5 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --actor 0 --e2e 0 --league-replay-extra 0 --e2e-5v5-extra 0"
for g in -1 0; do
for p in 0 1 0 1; do
  DCA_SIDE_PRIORITY=$p timeout -k 10 200 python -u bench.py $B --graph $g > gpurun_out/sp_$p.log 2>&1 || exit $?
  echo "graph $g prio $p $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sp_$p.log | head -1)" >> gpurun_out/sp_summary.txt
done
done
for p in 0 1 0 1; do
  DCA_SIDE_PRIORITY=$p timeout -k 10 200 python -u bench.py $B --model 5v5 --precision fp32 > gpurun_out/sp5_$p.log 2>&1 || exit $?
  echo "5v5 prio $p $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sp5_$p.log | head -1)" >> gpurun_out/sp_summary.txt
done

# exact learner step (and 5v5 step) with the graph-capture (main) stream at default vs high priority
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/mp_summary.txt
B="--steps 20 --warmup 5 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --actor 0 --e2e 0 --league-replay-extra 0 --e2e-5v5-extra 0"
for p in 0 1 0 1; do
  DCA_MAIN_PRIORITY=$p timeout -k 10 200 python -u bench.py $B > gpurun_out/mp_$p.log 2>&1 || exit $?
  echo "1v1 exact mainprio $p $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/mp_$p.log | head -1)" >> gpurun_out/mp_summary.txt
done
for p in 0 1; do
  DCA_MAIN_PRIORITY=$p timeout -k 10 200 python -u bench.py $B --precision fp32 > gpurun_out/mpb_$p.log 2>&1 || exit $?
  echo "1v1 bf16x3 mainprio $p $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/mpb_$p.log | head -1)" >> gpurun_out/mp_summary.txt
done
for p in 0 1; do
  DCA_MAIN_PRIORITY=$p timeout -k 10 200 python -u bench.py $B --model 5v5 --precision fp32 > gpurun_out/mp5_$p.log 2>&1 || exit $?
  echo "5v5 mainprio $p $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/mp5_$p.log | head -1)" >> gpurun_out/mp_summary.txt
done

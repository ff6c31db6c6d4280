# round 6 (i): hardware queues per process (GPU_MAX_HW_QUEUES, HIP default 4 on this pool) vs the two-policy
# pipelined actor step (two step streams sharing an in-order hardware queue serialise one's copies behind the other's
# kernels), then the node loops at both settings; the 5v5 weight-gradient GEMMs on two vs three streams
set -o pipefail
mkdir -p gpurun_out
for Q in 4 8; do
  for P in bf16 fp8 fp32; do
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python -u scripts/actor_bench.py 2048 $P > gpurun_out/r6i_actor_${P}_q$Q.json 2>&1 || exit $?
  done
done
E="--bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0"
timeout -k 10 600 python -u bench.py $E > gpurun_out/r6i_bench_q4.json 2> gpurun_out/r6i_bench_q4.err || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 600 python -u bench.py $E > gpurun_out/r6i_bench_q8.json 2> gpurun_out/r6i_bench_q8.err || exit $?
B5="--actor 0 --e2e 0 --league-replay-extra 0 --e2e-5v5-extra 0 --bptt350-extra 0 --big-batch-extra 0"
for R in a b; do
  for W in 1 2; do
    DCA_5V5_WG_BALANCE=$W timeout -k 10 400 python -u bench.py $B5 > gpurun_out/r6i_bench_bal${W}_$R.json 2> gpurun_out/r6i_bench_bal${W}_$R.err || exit $?
  done
done
echo done

# round 6 (r): the node loop's learner with the actor replaced by a CPU-only feeder process republishing synthetic raw
# rollouts (DCA_E2E_FEEDER=1: no actor kernels on the GPU) vs the real actor, same box — how much of the in-loop
# learner step (6.9-7.0 ms against 5.69 ms alone) is the actor's GPU work beside it
set -o pipefail
mkdir -p gpurun_out
E="--bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --league-replay-extra 0 --e2e-5v5-extra 0 --e2e-extra 0"
timeout -k 10 300 python -u bench.py $E > gpurun_out/r6r_bench_actor.json 2> gpurun_out/r6r_bench_actor.err || exit $?
DCA_E2E_FEEDER=1 timeout -k 10 300 python -u bench.py $E > gpurun_out/r6r_bench_feeder.json 2> gpurun_out/r6r_bench_feeder.err || exit $?
timeout -k 10 300 python -u bench.py $E > gpurun_out/r6r_bench_actor2.json 2> gpurun_out/r6r_bench_actor2.err || exit $?
DCA_E2E_FEEDER=1 timeout -k 10 300 python -u bench.py $E > gpurun_out/r6r_bench_feeder2.json 2> gpurun_out/r6r_bench_feeder2.err || exit $?
echo done

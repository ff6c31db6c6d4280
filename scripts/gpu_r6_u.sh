# round 6 (u): why the recurrence is slower in the node loop with nothing beside it — (a) sustained load: the learner
# step alone for 20 vs 1 500 back-to-back steps; (b) sequence packing (episode-start resets inside the recurrence):
# the feeder loop with and without packing
set -o pipefail
mkdir -p gpurun_out
L="--bf16x3-extra 0 --vtrace-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 0 --league-replay-extra 0 --e2e-5v5-extra 0"
timeout -k 10 300 python -u bench.py $L --steps 20 > gpurun_out/r6u_steps20.json 2> gpurun_out/r6u_steps20.err || exit $?
timeout -k 10 300 python -u bench.py $L --steps 1500 --warmup 5 > gpurun_out/r6u_steps1500.json 2> gpurun_out/r6u_steps1500.err || exit $?
E="--bf16x3-extra 0 --vtrace-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --league-replay-extra 0 --e2e-5v5-extra 0 --e2e-extra 0"
DCA_E2E_FEEDER=1 timeout -k 10 300 python -u bench.py $E --e2e-pack 0 > gpurun_out/r6u_feed_nopack.json 2> gpurun_out/r6u_feed_nopack.err || exit $?
DCA_E2E_FEEDER=1 timeout -k 10 300 python -u bench.py $E --e2e-pack 1 > gpurun_out/r6u_feed_pack.json 2> gpurun_out/r6u_feed_pack.err || exit $?
echo done

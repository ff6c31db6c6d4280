# round 6 (s): kernel traces of the node loop — with the CPU-only feeder (no actor kernels) and with the real actor
# process — learner idle gaps, per-call recurrence times (scripts/e2e_gaps.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
E="--steps 3 --warmup 1 --bf16x3-extra 0 --vtrace-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 8 --e2e-extra 0 --league-replay-extra 0 --e2e-5v5-extra 0"
rm -rf /tmp/prof_feed /tmp/prof_act
DCA_E2E_FEEDER=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_feed -- python3 bench.py $E > gpurun_out/r6s_feed.json 2> gpurun_out/r6s_feed.err || exit $?
python3 scripts/e2e_gaps.py /tmp/prof_feed --window-s 5 > gpurun_out/r6_e2e_gaps_feeder.txt 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_act -- python3 bench.py $E > gpurun_out/r6s_act.json 2> gpurun_out/r6s_act.err || exit $?
python3 scripts/e2e_gaps.py /tmp/prof_act --window-s 5 > gpurun_out/r6_e2e_gaps_actor.txt 2>&1 || exit $?
echo done
